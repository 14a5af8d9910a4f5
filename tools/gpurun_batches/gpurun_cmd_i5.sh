set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i5
mkdir -p $O
# the one-rank RCCL data-parallel step (--force-dp) next to the fused step on the current tree
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --force-dp --no-cpu-baseline > $O/fdp_$r.json 2> $O/fdp_$r.err &&
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/fused_$r.json 2> $O/fused_$r.err || exit 1
done &&
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_20_5.json 2> $O/fdp_20_5.err
echo "done $?"
