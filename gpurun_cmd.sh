set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/t_gpu_final.log 2>&1 &&
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o bench -- python3 -u bench.py > gpurun_out/prof_final.log 2>&1
echo "done $?"
