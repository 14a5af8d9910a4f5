#!/bin/bash
# round 6, batch l: the K-slice kernel with round 5's clean MFMA chain restored (asm fence in its own block + a
# sched_barrier behind the chain): parity of the top-layer kernels, launch-level A/B against round 5's kernel, the
# MLP3 step twice, a kernel trace of the step
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "affine_softmax or top or affine_fwd" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  $T 120 python3 tools/top_rows_bench.py > $O/top_new_$i.json 2> $O/top_new_$i.err &&
  TNET_LIB_VARIANT=oldtr $T 120 python3 tools/top_rows_bench.py > $O/top_old_$i.json 2> $O/top_old_$i.err || exit 1
done &&
$T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_1.json 2> $O/mlp3_1.err &&
$T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_2.json 2> $O/mlp3_2.err &&
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config mlp3 \
  --no-cpu-baseline --steps 300 --kernel-timing 0 > $O/prof.log 2>&1
rc=$?
echo "r6l rc=$rc"
exit $rc
