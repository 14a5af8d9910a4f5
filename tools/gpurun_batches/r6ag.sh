#!/bin/bash
# round 6, batch ag: the RNN weight updates (rnn_out_bwd's output-layer rows, the look-ahead launch's recurrent W)
# stored write-through -- RNN parity, then the frame chain against the library before the change (TNET_LIB_VARIANT=
# r6base) on one box
set -o pipefail
O=gpurun_out/r6ag
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rnn.py \
  tests/test_gpu_fullsize.py -k "rnn or Rnn or recurrent" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_LIB_VARIANT=r6base $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_base_$i.json 2> $O/rnn135_base_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_wt_$i.json 2> $O/rnn135_wt_$i.err &&
  TNET_LIB_VARIANT=r6base $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_base_$i.json 2> $O/rnn4000_base_$i.err &&
  $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_wt_$i.json 2> $O/rnn4000_wt_$i.err || exit 1
done
rc=$?
echo "r6ag rc=$rc"
exit $rc
