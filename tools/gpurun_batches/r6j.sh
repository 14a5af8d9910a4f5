#!/bin/bash
# round 6, batch j: why round 5's K-slice kernel ran 8.7 us and this round's 12.4 with the same MFMA / wait schedule --
# the only descriptor difference is the 9,352 B of LDS round 5's kernel declared (unused in the partials mode): the
# launch given that much dynamic LDS (TNET_TOP_ROWS_LDS) against none, against round 5's kernel, then the MLP3 step
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  for L in 0 9352 32768; do
    TNET_TOP_ROWS_LDS=$L $T 120 python3 tools/top_rows_bench.py > $O/top_lds${L}_$i.json 2> $O/top_lds${L}_$i.err || exit 1
  done
  TNET_LIB_VARIANT=oldtr $T 120 python3 tools/top_rows_bench.py > $O/top_oldtr_$i.json 2> $O/top_oldtr_$i.err || exit 1
done &&
for i in 1 2; do
  TNET_TOP_ROWS_LDS=0 $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_lds0_$i.json 2> $O/mlp3_lds0_$i.err &&
  TNET_TOP_ROWS_LDS=9352 $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_lds9352_$i.json \
    2> $O/mlp3_lds9352_$i.err || exit 1
done
rc=$?
echo "r6j rc=$rc"
exit $rc
