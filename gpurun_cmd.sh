set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests/test_ex01.py > gpurun_out/r3_ex01.log 2>&1 &&
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3_smoke.log 2>&1 &&
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_driverlike.json 2> gpurun_out/r3_bench_driverlike.err &&
timeout -k 10 300 python3 -u bench.py --config mlp3 > gpurun_out/r3_bench_mlp3.json 2> gpurun_out/r3_bench_mlp3.err &&
timeout -k 10 300 python3 -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err
echo "done $?"
