# MLP3 fused step: HIP API + kernel trace (is the 5-launch step host-bound? launch call times vs kernel times)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py \
  --config mlp3 --steps 40 --warmup 20 --no-cpu-baseline --breakdown-steps 0 > $O/bench.json 2> $O/bench.err
