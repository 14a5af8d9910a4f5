set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i13
mkdir -p $O
# the driver's 20 / 5 window with the 40-ms prewarm (default) vs without, interleaved; 100 / 20; the bench tests
timeout -k 10 400 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_bench.py -m gpu > $O/bench_tests.txt 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/pw_20_5_$r.json 2> $O/pw_20_5_$r.err &&
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --prewarm-ms 0 --no-cpu-baseline > $O/nopw_20_5_$r.json 2> $O/nopw_20_5_$r.err || exit 1
done &&
timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/pw_100_20.json 2> $O/pw_100_20.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/pw_20_5_cpu.json 2> $O/pw_20_5_cpu.err
echo "done $?"
