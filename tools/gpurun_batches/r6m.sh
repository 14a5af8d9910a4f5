#!/bin/bash
# round 6, batch m: (1) the 8-wave 64x64 configuration (m64x64k32s4w42: two waves a SIMD) -- GEMM parity over every
# configuration, then swept on the update / forward shapes of MLP3 and of dnn4's first layer against the 4-wave one;
# (2) round 5's whole library (lib/libtnet_amd_r05.so, TNET_LIB_VARIANT=r05) against this round's on one box:
# RNN 135 / 4000, MLP3, dnn4
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "gemm or affine" > $O/tests.txt 2>&1 &&
$T 600 python3 tools/gemm_sweep.py 40 auto,m64x64k32s4w41,m64x64k32s4w42 \
  '[["updb",1024,598,1024],["updb",1024,1024,135],["fwd",1024,598,1024],["updb",1024,440,2048],["fwd",1024,440,2048],["bwdcs",1024,1024,135]]' \
  > $O/sweep_w42.txt 2>&1 &&
for i in 1 2; do
  TNET_LIB_VARIANT=r05 $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_r05_$i.json 2> $O/rnn135_r05_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_r06_$i.json 2> $O/rnn135_r06_$i.err &&
  TNET_LIB_VARIANT=r05 $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_r05_$i.json 2> $O/rnn4000_r05_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_r06_$i.json 2> $O/rnn4000_r06_$i.err &&
  TNET_LIB_VARIANT=r05 $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_r05_$i.json 2> $O/mlp3_r05_$i.err &&
  $T 300 python3 bench.py --config mlp3 --no-cpu-baseline > $O/mlp3_r06_$i.json 2> $O/mlp3_r06_$i.err &&
  TNET_LIB_VARIANT=r05 $T 300 python3 bench.py --no-cpu-baseline > $O/dnn4_r05_$i.json 2> $O/dnn4_r05_$i.err &&
  $T 300 python3 bench.py --no-cpu-baseline > $O/dnn4_r06_$i.json 2> $O/dnn4_r06_$i.err || exit 1
done
rc=$?
echo "r6m rc=$rc"
exit $rc
