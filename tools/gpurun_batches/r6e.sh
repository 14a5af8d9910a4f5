#!/bin/bash
# round 6, batch e: the RNN look-ahead chain (TNET_RNN_AHEAD, one launch less a frame) -- RNN parity tests, then
# config 5 A/B interleaved at 135 and 4000 senones (tools/rnn_bench.py)
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rnn.py \
  tests/test_gpu_fullsize.py -k "rnn or Rnn or recurrent" > $O/tests.txt 2>&1 &&
for i in 1 2; do
  TNET_RNN_AHEAD=0 timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_off_$i.json 2> $O/rnn135_off_$i.err &&
  timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_on_$i.json 2> $O/rnn135_on_$i.err &&
  TNET_RNN_AHEAD=0 timeout -k 10 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_off_$i.json 2> $O/rnn4000_off_$i.err &&
  timeout -k 10 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_on_$i.json 2> $O/rnn4000_on_$i.err || exit 1
done
rc=$?
echo "r6e rc=$rc"
exit $rc
