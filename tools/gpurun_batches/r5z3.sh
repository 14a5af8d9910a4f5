# round-5 final tree: in-kernel GEMM clock stamps, the bench line again (it now reads profiles/r05_pmc_gemm2048.json
# for roofline.traffic), the driver's 20 / 5 window with and without the prewarm (two each), then the secondary
# configurations (tools/evidence_configs.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z3
mkdir -p $O
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2> $O/bench.err || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/window_prewarm_$r.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms 0 > $O/window_noprewarm_$r.json 2>> $O/bench.err || exit 1
done
bash tools/evidence_configs.sh
