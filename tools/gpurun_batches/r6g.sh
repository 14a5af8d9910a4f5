#!/bin/bash
# round 6, batch g: the data-parallel shadow apply reverted (parity re-run); the MLP3 top layer in the step
# (the K-slice kernel's loads fenced ahead of its MFMAs again) -- the combine / softmax kernel of this round (two rows a wave,
# parallel slab sums) against the previous one (lib/libtnet_amd_oldsx.so, TNET_LIB_VARIANT=oldsx), interleaved:
# the launch-level bench (tools/top_rows_bench.py) and the MLP3 bench line; then a kernel trace of the MLP3 step
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dp.py tests/test_gpu_shadow.py \
  tests/test_gpu_kernels.py -k "dp or shadow or affine_softmax or colsum or top or sgd" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  $T 120 python3 tools/top_rows_bench.py > $O/top_new_$i.json 2> $O/top_new_$i.err &&
  TNET_LIB_VARIANT=oldsx $T 120 python3 tools/top_rows_bench.py > $O/top_old_$i.json 2> $O/top_old_$i.err &&
  $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_new_$i.json 2> $O/mlp3_new_$i.err &&
  TNET_LIB_VARIANT=oldsx $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_old_$i.json \
    2> $O/mlp3_old_$i.err || exit 1
done &&
$T 300 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run -- python3 bench.py --config mlp3 --no-cpu-baseline \
  --steps 300 --kernel-timing 0 > $O/prof_new.log 2>&1 &&
TNET_LIB_VARIANT=oldsx $T 300 rocprofv3 --kernel-trace --stats -d $O/prof_old -o run -- python3 bench.py --config mlp3 \
  --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof_old.log 2>&1
rc=$?
echo "r6g rc=$rc"
exit $rc
