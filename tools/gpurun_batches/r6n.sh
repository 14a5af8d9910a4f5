#!/bin/bash
# round 6, batch n: which RNN kernels changed between round 5's library and this round's -- kernel traces of the frame
# chain, both libraries, 135 and 4000 senones (tools/rnn_frame_trace.py; TNET_RNN_AHEAD=0 and default for this round)
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for S in 135 4000; do
  TNET_LIB_VARIANT=r05 $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/r05_$S -o run -- python3 \
    tools/rnn_frame_trace.py run $S > $O/r05_$S.log 2>&1 &&
  TNET_RNN_AHEAD=0 $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/r06off_$S -o run -- python3 \
    tools/rnn_frame_trace.py run $S > $O/r06off_$S.log 2>&1 &&
  $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/r06_$S -o run -- python3 tools/rnn_frame_trace.py run $S \
    > $O/r06_$S.log 2>&1 || exit 1
done
rc=$?
echo "r6n rc=$rc"
exit $rc
