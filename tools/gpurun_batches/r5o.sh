# tile-configuration sweep over the small-K shapes: MLP3's first layer (K = 598) and dnn4's (K = 440)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 600 python3 tools/gemm_sweep.py 50 \
  auto,m64x64k32s4w41,m64x64k64s2,m64x64k32s4,m32x64k64s2,m64x128k64s2,m64x128k32s4,m64x128a8,m64x128a4,m64x128d4,m128x128a4,g64x64k32s4w4 \
  '[["fwd",1024,598,1024],["updb",1024,598,1024],["fwd",1024,440,2048],["updb",1024,440,2048]]' > $O/sweep.txt 2>&1
