#!/bin/bash
# round 6, batch s (diagnosis, timing only): the look-ahead first launch with its update workgroups dropped
# (TNET_DIAG_NO_RNN_UPD=1: results wrong, times right) against the full launch -- is the update or the correction path
# the 1.5 us over round 5's 5.8 us?
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
for S in 135 4000; do
  TNET_DIAG_NO_RNN_UPD=1 $T 240 rocprofv3 --kernel-trace --output-format csv -d $O/noupd_$S -o run -- python3 \
    tools/rnn_frame_trace.py run $S > $O/noupd_$S.log 2>&1 || exit 1
done
rc=$?
echo "r6s rc=$rc"
exit $rc
