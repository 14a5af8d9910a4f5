# the driver's 20 / 5 window with the default 200 ms prewarm vs 400 ms and 800 ms, interleaved x4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z13
mkdir -p $O
for r in 1 2 3 4; do
  for ms in 200 400 800; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms $ms > $O/w${ms}_$r.json 2>> $O/err.txt || exit 1
  done
done
