# DP exchange schedule: the step's whole reduction inline on the compute stream (MLP3) and the applies on the comm
# stream (dnn4): DP tests, then force-dp A/B benches interleaved (TNET_DP_INLINE / TNET_DP_APPLY_COMM)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dp.py \
  tests/test_gpu_bench.py > $O/tests.txt 2>&1 || exit 1
B="--no-cpu-baseline --breakdown-steps 0"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 400 --warmup 50 $B > $O/mlp3_fdp_new_$r.json 2>> $O/bench.err || exit 1
  TNET_DP_INLINE=0 TNET_DP_APPLY_COMM=0 timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 400 --warmup 50 $B \
    > $O/mlp3_fdp_old_$r.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --config mlp3 --steps 400 --warmup 50 $B > $O/mlp3_fused_$r.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --force-dp --steps 100 --warmup 20 $B > $O/dnn4_fdp_new_$r.json 2>> $O/bench.err || exit 1
  TNET_DP_APPLY_COMM=0 timeout -k 10 200 python3 bench.py --force-dp --steps 100 --warmup 20 $B > $O/dnn4_fdp_old_$r.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 $B > $O/dnn4_fused_$r.json 2>> $O/bench.err || exit 1
done
