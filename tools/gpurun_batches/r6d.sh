#!/bin/bash
# round 6, batch d: the step's last two updates balanced over one round (gemm16_upd_balanced_kernel) with the next
# bunch's gather riding on the softmax launch -- parity tests, then dnn4 A/B interleaved:
#   base = TNET_GATHER_SOFTMAX=0 (round 5: gather on the mixed last-update launch), new = default,
#   sep  = TNET_UPD_BALANCED=0 (gather on the softmax, the two updates as separate launches)
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "update_bias_pair or softmax_xent_gather or update_bias_gather" \
  tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_shadow.py tests/test_gpu_recovery.py \
  > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_GATHER_SOFTMAX=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/base_$i.json 2> $O/base_$i.err &&
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/new_$i.json 2> $O/new_$i.err &&
  TNET_UPD_BALANCED=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/sep_$i.json 2> $O/sep_$i.err || exit 1
done &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/new_20_5.json 2> $O/new_20_5.err
rc=$?
echo "r6d rc=$rc"
exit $rc
