set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i7
mkdir -p $O
# the exchange's events without the system-scope fence (default) vs with it (TNET_DP_EVENT_FENCE=1): the DP
# tests, then the one-rank RCCL step interleaved, then a kernel trace of the new default
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_dp.py -m gpu > $O/dp_tests.txt 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --force-dp --no-cpu-baseline > $O/nofence_$r.json 2> $O/nofence_$r.err &&
  TNET_DP_EVENT_FENCE=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --force-dp --no-cpu-baseline > $O/fence_$r.json 2> $O/fence_$r.err || exit 1
done &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/nofence_20_5.json 2> $O/nofence_20_5.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o fdp -- python3 bench.py --steps 30 --warmup 10 --force-dp --no-cpu-baseline > $O/fdp_prof.json 2> $O/fdp_prof.err
echo "done $?"
