#!/bin/bash
# round 6, batch aa: the MLP3 combine / softmax kernel with every load in one round (labels, slice 0, bias and the
# other slices at clamped indices behind a fence) against the previous build (TNET_LIB_VARIANT=prev) -- parity of the
# top-layer kernels and the MLP3 training tests, launch-level and step A/B, a kernel trace of each
set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_train.py tests/test_gpu_fullsize.py -k "affine_softmax or colsum or mlp or MLP or top or softmax" \
  > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_LIB_VARIANT=prev $T 120 python3 tools/top_rows_bench.py > $O/top_prev_$i.json 2> $O/top_prev_$i.err &&
  $T 120 python3 tools/top_rows_bench.py > $O/top_new_$i.json 2> $O/top_new_$i.err &&
  TNET_LIB_VARIANT=prev $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_prev_$i.json 2> $O/mlp3_prev_$i.err &&
  $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_new_$i.json 2> $O/mlp3_new_$i.err || exit 1
done &&
for v in prev new; do
  if [ $v = new ]; then unset TNET_LIB_VARIANT; else export TNET_LIB_VARIANT=prev; fi
  $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --config mlp3 \
    --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof_$v.log 2>&1 || exit 1
done
rc=$?
echo "r6aa rc=$rc"
exit $rc
