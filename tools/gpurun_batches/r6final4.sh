#!/bin/bash
# round 6, closing check on the committed tree (after the RNN write-through weight updates): the whole GPU suite, smoke(), the driver's default bench command and
# its 20 / 5 window
set -o pipefail
O=gpurun_out/final4
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.txt 2>&1 &&
$T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
$T 420 python3 bench.py > $O/bench.json 2> $O/bench.err &&
$T 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_window.json 2> $O/bench_window.err
rc=$?
echo "final4 rc=$rc"
exit $rc
