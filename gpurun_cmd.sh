set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3s3_gpu_suite_last.txt 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3s3_smoke_last.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r3s3_bench_window_last.json 2> gpurun_out/r3s3_bench_window_last.err
echo "done $?"
