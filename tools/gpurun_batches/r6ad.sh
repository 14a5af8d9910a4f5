#!/bin/bash
# round 6, batch ad: the next frame's recurrent output finished by the last BPTT launch (tnet_gemv_rows_hnext) --
# RNN parity (incl. bit-identity against TNET_RNN_HNEXT=0), then the frame chain on vs off on one box, and a kernel
# trace of each size
set -o pipefail
O=gpurun_out/r6ad
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rnn.py \
  tests/test_gpu_fullsize.py -k "rnn or Rnn or recurrent" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_RNN_HNEXT=0 $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_off_$i.json 2> $O/rnn135_off_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_on_$i.json 2> $O/rnn135_on_$i.err &&
  TNET_RNN_HNEXT=0 $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_off_$i.json 2> $O/rnn4000_off_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_on_$i.json 2> $O/rnn4000_on_$i.err || exit 1
done &&
for S in 135 4000; do
  $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/on_$S -o run -- python3 tools/rnn_frame_trace.py run $S \
    > $O/on_$S.log 2>&1 || exit 1
done
rc=$?
echo "r6ad rc=$rc"
exit $rc
