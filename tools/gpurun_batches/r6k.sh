#!/bin/bash
# round 6, batch k: bisecting the MLP3 K-slice kernel's 12.4 vs 8.7 us in the step -- kernel traces of the MLP3 bench
# with this round's kernel (default), round 5's (oldtr), this round's with round 5's 200-byte kernarg (trB), round 5's
# without its clock-stamp code (trC)
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for v in default oldtr trB trC; do
  if [ $v = default ]; then unset TNET_LIB_VARIANT; else export TNET_LIB_VARIANT=$v; fi
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --config mlp3 \
    --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof_$v.log 2>&1 || exit 1
done
rc=$?
echo "r6k rc=$rc"
exit $rc
