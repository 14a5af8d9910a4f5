#!/bin/bash
# round 6, batch ae: HIP runtime launch knobs on the launch-bound RNN frame chain (graph replay of 96-frame
# segments): default vs device-memory kernel arguments vs the graph packet-capture path on / off, two runs each
set -o pipefail
O=gpurun_out/r6ae
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for i in 1 2; do
  $T 300 python3 tools/rnn_bench.py 4 135 > $O/def_$i.json 2> $O/def_$i.err &&
  HIP_FORCE_DEV_KERNARG=1 $T 300 python3 tools/rnn_bench.py 4 135 > $O/devka_$i.json 2> $O/devka_$i.err &&
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $T 300 python3 tools/rnn_bench.py 4 135 > $O/pc0_$i.json 2> $O/pc0_$i.err &&
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 $T 300 python3 tools/rnn_bench.py 4 135 > $O/pc1_$i.json 2> $O/pc1_$i.err || exit 1
done
rc=$?
echo "r6ae rc=$rc"
exit $rc
