#!/bin/bash
# round 6, batch z: the forward kernel specialised on the look-ahead form at compile time (template<bool>)
# vectorised, the correction's d_i and the slice dots in one round) -- RNN parity, then the frame chain against round
# 5's library on one box, and a kernel trace of each
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rnn.py \
  tests/test_gpu_fullsize.py -k "rnn or Rnn or recurrent" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_LIB_VARIANT=r05 $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_r05_$i.json 2> $O/rnn135_r05_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_r06_$i.json 2> $O/rnn135_r06_$i.err &&
  TNET_LIB_VARIANT=r05 $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_r05_$i.json 2> $O/rnn4000_r05_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_r06_$i.json 2> $O/rnn4000_r06_$i.err || exit 1
done &&
for S in 135 4000; do
  $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/r06_$S -o run -- python3 tools/rnn_frame_trace.py run $S \
    > $O/r06_$S.log 2>&1 || exit 1
done
rc=$?
echo "r6z rc=$rc"
exit $rc
