set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i2
mkdir -p $O
# the whole GPU suite on the TNET_GEMM_KC=1 default (c8 for the top layer's backward only), then the SGD step
# KC=1 / KC=0 interleaved and the driver's 20 / 5 window
timeout -k 10 700 python3 -u -m pytest tests -x -q -rf -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1 &&
for r in 1 2; do
  TNET_GEMM_KC=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/kc1_$r.json 2> $O/kc1_$r.err &&
  TNET_GEMM_KC=0 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/kc0_$r.json 2> $O/kc0_$r.err || exit 1
done &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_20_5.json 2> $O/bench_20_5.err
echo "done $?"
