# where the MLP3 one-rank DP step's time goes: kernel trace (+ HIP runtime API trace, no counters) of the
# force-dp step, fused step beside it; the per-step gaps between kernels read from the trace databases
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z14
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/fdp -o run -- python3 bench.py --config mlp3 --force-dp --no-cpu-baseline --steps 200 --warmup 20 --kernel-timing 0 --breakdown-steps 0 --prewarm-ms 0 > $O/fdp.json 2> $O/fdp.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/fused -o run -- python3 bench.py --config mlp3 --no-cpu-baseline --steps 200 --warmup 20 --kernel-timing 0 --breakdown-steps 0 --prewarm-ms 0 > $O/fused.json 2> $O/fused.err
