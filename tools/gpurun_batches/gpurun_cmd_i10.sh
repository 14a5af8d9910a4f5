set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i10
mkdir -p $O
# MLP3 data-parallel lines on the fence-free exchange events (default) vs the fence (TNET_DP_EVENT_FENCE=1)
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_fdp_$r.json 2> $O/mlp3_fdp_$r.err &&
  TNET_DP_EVENT_FENCE=1 timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_fdp_fence_$r.json 2> $O/mlp3_fdp_fence_$r.err &&
  timeout -k 10 200 python3 bench.py --config mlp3 --bunch 128 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_b128_fdp_$r.json 2> $O/mlp3_b128_fdp_$r.err &&
  TNET_DP_EVENT_FENCE=1 timeout -k 10 200 python3 bench.py --config mlp3 --bunch 128 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_b128_fdp_fence_$r.json 2> $O/mlp3_b128_fdp_fence_$r.err || exit 1
done &&
timeout -k 10 200 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_fused.json 2> $O/mlp3_fused.err &&
timeout -k 10 200 python3 bench.py --config mlp3 --bunch 128 --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_b128_fused.json 2> $O/mlp3_b128_fused.err
echo "done $?"
