#!/bin/bash
# round 6, batch t: where the one-rank data-parallel step's extra 6 % goes -- kernel traces (with per-dispatch
# timestamps) of the dnn4 fused step and of the --force-dp step, 100 steps each
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fused -o run -- python3 bench.py --no-cpu-baseline \
  --kernel-timing 0 > $O/fused.json 2> $O/fused.err &&
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dp -o run -- python3 bench.py --force-dp \
  --no-cpu-baseline --kernel-timing 0 > $O/dp.json 2> $O/dp.err
rc=$?
echo "r6t rc=$rc"
exit $rc
