set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i14
mkdir -p $O
# the prewarm length on the driver's 20 / 5 window
for r in 1 2; do
  for ms in 40 100 200; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --prewarm-ms $ms --no-cpu-baseline > $O/pw${ms}_$r.json 2> $O/pw${ms}_$r.err || exit 1
  done
done
echo "done $?"
