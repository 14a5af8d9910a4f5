# round-5 final tree (after the softmax label-first change), final evidence: tools/profile_round.sh (bench line with the CPU baseline, rocprofv3 stats of the
# same command, FETCH / WRITE / MFMA PMC passes, GEMM clock stamps), then the driver's 20 / 5 window with the default
# prewarm and cold, two each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh || exit 1
O=gpurun_out/r5z10
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/window_$r.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms 0 > $O/window_cold_$r.json 2>> $O/bench.err || exit 1
done
