set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i11
mkdir -p $O
# the driver's 20 / 5 window against longer warm-ups / windows, same box
for cfg in "20 5" "20 20" "40 5" "100 5" "100 20" "20 5"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline > $O/w_$1_$2_$RANDOM.json 2> $O/w_$1_$2.err || exit 1
done
echo "done $?"
