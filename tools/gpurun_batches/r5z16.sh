# the next pass's permutation drawn ahead on a host thread (CuCache, TNET_SHUFFLE_AHEAD): MLP3 fused / one-rank DP
# and dnn4 A/B interleaved, host_rate for MLP3 DP, then the whole GPU suite and smoke()
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z16
mkdir -p $O
for r in 1 2 3; do
  for a in 1 0; do
    TNET_SHUFFLE_AHEAD=$a timeout -k 10 200 python3 bench.py --config mlp3 --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3_a${a}_$r.json 2>> $O/err.txt || exit 1
    TNET_SHUFFLE_AHEAD=$a timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3fdp_a${a}_$r.json 2>> $O/err.txt || exit 1
  done
done
for r in 1 2; do
  for a in 1 0; do
    TNET_SHUFFLE_AHEAD=$a timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/dnn4_a${a}_$r.json 2>> $O/err.txt || exit 1
  done
done
timeout -k 10 200 python3 tools/host_rate.py --config mlp3 --force-dp --steps 640 > $O/host_fdp.json 2>> $O/err.txt &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
