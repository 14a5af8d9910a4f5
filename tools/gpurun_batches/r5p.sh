# the driver's 20 / 5 window: prewarm forms A/B (scratch training steps vs scratch GEMMs vs none), interleaved,
# two rounds, then the 100 / 20 line with the steps form
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5p
mkdir -p $O
for r in 1 2; do
  for f in steps gemm; do
    timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --prewarm-form $f > $O/w_${f}_$r.json 2>> $O/bench.err || exit 1
  done
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms 0 > $O/w_none_$r.json 2>> $O/bench.err || exit 1
done
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/default_steps.json 2>> $O/bench.err
