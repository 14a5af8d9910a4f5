set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i9
mkdir -p $O
# WaitAll without its comm-stream wait when the compute / apply stream already covered the comm stream (default)
# vs always (TNET_DP_WAITALL_COMM=1), and the last layer's apply on the apply stream (TNET_DP_LAST_APPLY_STREAM=1)
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_dp.py -m gpu > $O/dp_tests.txt 2>&1 &&
TNET_DP_LAST_APPLY_STREAM=1 timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_dp.py -m gpu > $O/dp_tests_lastapply.txt 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --force-dp --no-cpu-baseline > $O/skip_$r.json 2> $O/skip_$r.err &&
  TNET_DP_WAITALL_COMM=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --force-dp --no-cpu-baseline > $O/always_$r.json 2> $O/always_$r.err &&
  TNET_DP_LAST_APPLY_STREAM=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --force-dp --no-cpu-baseline > $O/lastapply_$r.json 2> $O/lastapply_$r.err || exit 1
done &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/skip_20_5.json 2> $O/skip_20_5.err
echo "done $?"
