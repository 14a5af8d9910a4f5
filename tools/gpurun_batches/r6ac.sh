#!/bin/bash
# round 6, batch ac: the unarmed record of block sizes bounded to the latest step -- the
# DP / bench suites, then the armed steps' HIP trace again (tools/armed_step_trace.py)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r6ac
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench.py \
  tests/test_gpu_dp.py > gpurun_out/r6ac/tests.txt 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --hip-trace --marker-trace --output-format csv -d "$R/gpurun_out/r6ac/armed" -o armed \
  -- python3 "$R/tools/armed_step_trace.py" run > "$R/gpurun_out/r6ac/armed_run.json" 2> "$R/gpurun_out/r6ac/armed_run.err" &&
cd "$R" &&
python3 tools/armed_step_trace.py summarize gpurun_out/r6ac/armed > gpurun_out/r6ac/armed_summary.json
rc=$?
echo "r6ac rc=$rc"
exit $rc
