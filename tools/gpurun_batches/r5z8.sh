# the softmax change (r5z7) again: dnn4 bench A/B interleaved x5 (old first in each pair this time), 300 steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z8
mkdir -p $O
for r in 1 2 3 4 5; do
  TNET_LIB_VARIANT=smold timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 300 --warmup 20 > $O/old_$r.json 2>> $O/err.txt || exit 1
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 300 --warmup 20 > $O/new_$r.json 2>> $O/err.txt || exit 1
done
