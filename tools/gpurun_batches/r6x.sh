#!/bin/bash
# round 6, batch x: is the 64x64 direct form worth making the MLP3 updates eligible (M = 598 fails its M % 4 rule;
# 160 tiles its 200-tile rule)? The same updates at n_in 600 / n_out 136 (eligible shapes) under the ring and the
# direct forms; then the drop-in tests after the drop-in relink
set -o pipefail
O=gpurun_out/r6x
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 tools/gemm_sweep.py 40 auto,m64x64k32s4w41,m64x64a4 \
  '[["updb",1024,598,1024],["updb",1024,600,1024],["updb",1024,1024,135],["updb",1024,1024,136],["updb",1024,440,2048]]' \
  > $O/sweep_direct.txt 2>&1 &&
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dropin.py > $O/dropin.txt 2>&1
rc=$?
echo "r6x rc=$rc"
exit $rc
