# round-5 final tree: the metric-config evidence (tools/profile_round.sh: bench line with the CPU baseline, rocprofv3
# kernel-trace stats of the same command, FETCH / WRITE / MFMA PMC passes), then the driver's 20 / 5 window with and
# without the prewarm, two runs each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/profile_round.sh || exit 1
O=gpurun_out/r5z2
mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/window_prewarm_$r.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --prewarm-ms 0 > $O/window_noprewarm_$r.json 2>> $O/bench.err || exit 1
done
