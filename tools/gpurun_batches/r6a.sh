#!/bin/bash
# round 6, batch a: the ADVICE r5 shadow fixes, the device-side reduction-check capture, the
# one-rank swap rehearsal; the armed step's HIP trace; the force-dp line with the N > 1 CU reservation (item 2)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r6a
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shadow.py \
  tests/test_gpu_bench.py tests/test_gpu_dp.py > gpurun_out/r6a/tests.txt 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --hip-trace --marker-trace --output-format csv -d "$R/gpurun_out/r6a/armed" -o armed \
  -- python3 "$R/tools/armed_step_trace.py" run > "$R/gpurun_out/r6a/armed_run.json" 2> "$R/gpurun_out/r6a/armed_run.err" &&
cd "$R" &&
python3 tools/armed_step_trace.py summarize gpurun_out/r6a/armed > gpurun_out/r6a/armed_summary.json &&
timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6a/forcedp.json 2> gpurun_out/r6a/forcedp.err &&
TNET_DP_RESERVE_CUS=16 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6a/forcedp_res16.json 2> gpurun_out/r6a/forcedp_res16.err &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r6a/fused.json 2> gpurun_out/r6a/fused.err &&
TNET_DP_RESERVE_CUS=16 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6a/forcedp_res16_b.json 2> gpurun_out/r6a/forcedp_res16_b.err &&
timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6a/forcedp_b.json 2> gpurun_out/r6a/forcedp_b.err
rc=$?
echo "r6a rc=$rc"
exit $rc
