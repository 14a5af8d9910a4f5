#!/bin/bash
# round 6, batch f: (1) parity of the changed kernels -- the MLP3 top kernel (two rows a wave, parallel slab sums),
# the shadow-keeping data-parallel apply (tnet_sgd_update_multi_t) and the DP / shadow suites; (2) the data-parallel
# step at one rank with the shadow kept vs not (TNET_DP_SHADOW=0), plain and with 16 CUs reserved (the N = 8
# backward's grid); (3) MLP3: the config sweep of its shapes, the top layer's launches, two bench lines
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "affine_softmax or colsum or softmax or sgd_update" > $O/tests_kernels.txt 2>&1 &&
$T 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dp.py \
  tests/test_gpu_shadow.py tests/test_gpu_train.py > $O/tests_dp.txt 2>&1 &&
for i in 1 2; do
  $T 300 python3 bench.py --force-dp --no-cpu-baseline > $O/dp_shadow_$i.json 2> $O/dp_shadow_$i.err &&
  TNET_DP_SHADOW=0 $T 300 python3 bench.py --force-dp --no-cpu-baseline > $O/dp_flat_$i.json 2> $O/dp_flat_$i.err &&
  TNET_DP_RESERVE_CUS=16 $T 300 python3 bench.py --force-dp --no-cpu-baseline > $O/dp_res16_shadow_$i.json \
    2> $O/dp_res16_shadow_$i.err &&
  TNET_DP_SHADOW=0 TNET_DP_RESERVE_CUS=16 $T 300 python3 bench.py --force-dp --no-cpu-baseline \
    > $O/dp_res16_flat_$i.json 2> $O/dp_res16_flat_$i.err &&
  $T 300 python3 bench.py --no-cpu-baseline > $O/fused_$i.json 2> $O/fused_$i.err || exit 1
done &&
$T 900 python3 tools/gemm_sweep.py 40 \
  auto,m64x64k32s4w41,m64x64a4,m64x64k64s2,m64x64k32s4,m32x64k64s2,m64x128k64s2,m64x128a4,g64x64k32s4w4 \
  '[["fwd",1024,598,1024],["updb",1024,598,1024],["bwdcs",1024,1024,135],["updb",1024,1024,135]]' \
  > $O/sweep_mlp3.txt 2>&1 &&
$T 300 python3 tools/top_rows_bench.py > $O/top_rows.json 2> $O/top_rows.err &&
$T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_1.json 2> $O/mlp3_1.err &&
$T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_2.json 2> $O/mlp3_2.err
rc=$?
echo "r6f rc=$rc"
exit $rc
