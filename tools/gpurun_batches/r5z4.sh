# with the wide pair on: the top layer's shadow (TNET_BWD_SHADOW=1: every layer) vs hidden layers only (2, default),
# dnn4 interleaved x3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z4
mkdir -p $O
for r in 1 2 3; do
  for m in 1 2; do
    TNET_BWD_SHADOW=$m timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/dnn4_s${m}_$r.json 2>> $O/bench.err || exit 1
  done
done
