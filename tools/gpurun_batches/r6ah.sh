#!/bin/bash
# round 6, batch ah: the RBM sampling epilogue's states and generator state stored write-through -- RBM parity, then
# the CD-1 step against the library before the change (TNET_LIB_VARIANT=r6base) on one box, bunch 256 and 1024
set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rbm.py \
  tests/test_gpu_fullsize.py -k "rbm or Rbm" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_LIB_VARIANT=r6base $T 300 python3 tools/rbm_bench.py 256 2000 1 > $O/rbm256_base_$i.json 2> $O/rbm256_base_$i.err &&
  $T 300 python3 tools/rbm_bench.py 256 2000 1 > $O/rbm256_wt_$i.json 2> $O/rbm256_wt_$i.err &&
  TNET_LIB_VARIANT=r6base $T 300 python3 tools/rbm_bench.py 1024 1000 1 > $O/rbm1024_base_$i.json 2> $O/rbm1024_base_$i.err &&
  $T 300 python3 tools/rbm_bench.py 1024 1000 1 > $O/rbm1024_wt_$i.json 2> $O/rbm1024_wt_$i.err || exit 1
done
rc=$?
echo "r6ah rc=$rc"
exit $rc
