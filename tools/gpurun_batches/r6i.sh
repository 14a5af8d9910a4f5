#!/bin/bash
# round 6, batch i: the MLP3 top layer's K-slice kernel of this round (loads fenced ahead of the MFMAs) against round
# 5's (lib/libtnet_amd_oldtr.so: its row-block kernel in the partials mode, TNET_LIB_VARIANT=oldtr), interleaved --
# launch-level (tools/top_rows_bench.py), in the step (bench.py --config mlp3) and under a kernel trace
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 120 python3 tools/top_rows_bench.py > $O/top_new_$i.json 2> $O/top_new_$i.err &&
  TNET_LIB_VARIANT=oldtr $T 120 python3 tools/top_rows_bench.py > $O/top_old_$i.json 2> $O/top_old_$i.err &&
  $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_new_$i.json 2> $O/mlp3_new_$i.err &&
  TNET_LIB_VARIANT=oldtr $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_old_$i.json \
    2> $O/mlp3_old_$i.err || exit 1
done &&
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python3 bench.py --config mlp3 \
  --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof_new.log 2>&1 &&
TNET_LIB_VARIANT=oldtr $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_old -o run -- python3 \
  bench.py --config mlp3 --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof_old.log 2>&1
rc=$?
echo "r6i rc=$rc"
exit $rc
