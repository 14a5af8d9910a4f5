# MLP3 one-rank data-parallel step (bench --force-dp) vs the fused step: kernel traces for the step timeline (where
# the DP path's extra ~40 us go), then the r5d throughput benches (bunch 128..1024, force-dp and fused)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5i
mkdir -p $O
for m in fdp fused; do
  f=""; [ $m = fdp ] && f="--force-dp"
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$m -o run -- python3 bench.py --config mlp3 \
    $f --steps 40 --warmup 20 --no-cpu-baseline --breakdown-steps 0 > $O/bench_$m.json 2> $O/bench_$m.err || exit 1
done
bash tools/gpurun_batches/r5d.sh bench
