#!/bin/bash
# round 6, batch h: (1) where an RNN frame's time goes -- kernel traces of the fused frame chain (look-ahead on) at
# 135 and 4000 senones, summarized per kernel kind with the idle gap before each (tools/rnn_frame_trace.py);
# (2) the MLP3 one-rank DP step at 256 and 1024 rows a rank
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for S in 135 4000; do
  $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/rnn$S -o run -- python3 tools/rnn_frame_trace.py run $S \
    > $O/rnn${S}_run.log 2>&1 || exit 1
done &&
for B in 256 1024; do
  $T 300 python3 bench.py --config mlp3 --force-dp --bunch $B --no-cpu-baseline > $O/mlp3_dp_b$B.json \
    2> $O/mlp3_dp_b$B.err &&
  $T 300 python3 bench.py --config mlp3 --bunch $B --no-cpu-baseline > $O/mlp3_b$B.json 2> $O/mlp3_b$B.err || exit 1
done
rc=$?
echo "r6h rc=$rc"
exit $rc
