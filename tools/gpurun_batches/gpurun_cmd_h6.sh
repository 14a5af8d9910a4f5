set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h6
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 &&
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock.log 2>&1
echo "done $?"
