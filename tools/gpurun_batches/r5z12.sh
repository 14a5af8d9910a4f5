# round-5 final tree after the wave-per-row softmax's label-first form and the stamp-clear ordering fix: the whole
# GPU suite, smoke(), then the GEMM clock stamps twice (the fix: no workgroup's first stamps lost under the clear)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z12
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock_1.log 2>&1 &&
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock_2.log 2>&1
