#!/bin/bash
# round 6, batch b: the whole GPU suite on the pruned library (the dead-end forms removed: VERDICT r5 item 7), the
# armed step's HIP trace (item 1), the force-dp line with and without the N > 1 CU reservation (item 2)
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r6b
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r6b/gpu_suite.txt 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --hip-trace --marker-trace --output-format csv -d "$R/gpurun_out/r6b/armed" -o armed \
  -- python3 "$R/tools/armed_step_trace.py" run > "$R/gpurun_out/r6b/armed_run.json" 2> "$R/gpurun_out/r6b/armed_run.err" &&
cd "$R" &&
{ python3 tools/armed_step_trace.py summarize gpurun_out/r6b/armed > gpurun_out/r6b/armed_summary.json; true; } &&
timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6b/forcedp.json 2> gpurun_out/r6b/forcedp.err &&
TNET_DP_RESERVE_CUS=16 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6b/forcedp_res16.json 2> gpurun_out/r6b/forcedp_res16.err &&
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r6b/fused.json 2> gpurun_out/r6b/fused.err &&
TNET_DP_RESERVE_CUS=16 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6b/forcedp_res16_b.json 2> gpurun_out/r6b/forcedp_res16_b.err &&
timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > gpurun_out/r6b/forcedp_b.json 2> gpurun_out/r6b/forcedp_b.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --no-cpu-baseline > gpurun_out/r6b/mlp3.json 2> gpurun_out/r6b/mlp3.err
rc=$?
echo "r6b rc=$rc"
exit $rc
