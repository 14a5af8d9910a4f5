#!/bin/bash
# round 6, batch ab: the RNN frame chain's hipGraph segment length (TNET_RNN_GRAPH_FRAMES: 96 default) -- 96 vs 160 vs
# 320 frames a segment, interleaved, 135 and 4000 senones
set -o pipefail
O=gpurun_out/r6ab
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  for F in 96 160 320; do
    TNET_RNN_GRAPH_FRAMES=$F $T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_f${F}_$i.json 2> $O/rnn135_f${F}_$i.err &&
    TNET_RNN_GRAPH_FRAMES=$F $T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_f${F}_$i.json 2> $O/rnn4000_f${F}_$i.err || exit 1
  done
done
rc=$?
echo "r6ab rc=$rc"
exit $rc
