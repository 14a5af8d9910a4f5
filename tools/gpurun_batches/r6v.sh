#!/bin/bash
# round 6, batch v: MLP3's K = 598 first-layer forward and the 1024 x 135 update under split-K (TNET_GEMM_SPLITK: the
# slices combined by the split-K reduce with the bias + sigmoid / SGD epilogue) against the one-slice plan
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/gemm_sweep.py 40 \
  auto,m64x64k32s4w41+sk2,m64x64k32s4w41+sk3,m64x64k64s2+sk2,m32x64k64s2+sk2,m64x128k64s2+sk2,m128x128k64s2+sk4 \
  '[["fwd",1024,598,1024],["updb",1024,598,1024],["updb",1024,1024,135]]' > $O/sweep_sk.txt 2>&1
rc=$?
echo "r6v rc=$rc"
exit $rc
