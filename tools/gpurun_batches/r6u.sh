#!/bin/bash
# round 6, batch u: the MLP3 combine kernel's slab column sums in 8 parallel row groups (lib/libtnet_amd_cs.so,
# TNET_LIB_VARIANT=cs) against the 32-deep chain (default lib) -- parity of the top-layer kernels with the variant, then
# interleaved launch-level and step A/B, and a kernel trace of each
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
TNET_LIB_VARIANT=cs $T 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_train.py -k "affine_softmax or colsum or mlp or MLP or top" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  $T 120 python3 tools/top_rows_bench.py > $O/top_old_$i.json 2> $O/top_old_$i.err &&
  TNET_LIB_VARIANT=cs $T 120 python3 tools/top_rows_bench.py > $O/top_cs_$i.json 2> $O/top_cs_$i.err &&
  $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_old_$i.json 2> $O/mlp3_old_$i.err &&
  TNET_LIB_VARIANT=cs $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_cs_$i.json 2> $O/mlp3_cs_$i.err || exit 1
done &&
for v in old cs; do
  if [ $v = old ]; then unset TNET_LIB_VARIANT; else export TNET_LIB_VARIANT=cs; fi
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --config mlp3 \
    --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof_$v.log 2>&1 || exit 1
done
rc=$?
echo "r6u rc=$rc"
exit $rc
