#!/bin/bash
# round 6, batch c: the top layer's forward-written transposed shadow (f4 form, tnet_affine_fwd_shadow) -- its
# parity tests, then the whole GPU suite on the pruned library; the armed step's HIP trace;
# dnn4 A/B of the forward shadow (TNET_FWD_SHADOW=0/1, interleaved); the force-dp lines with / without the N > 1 CU
# reservation (item 2)
set -o pipefail
R=$(pwd)
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_shadow.py \
  > $O/shadow_tests.txt 2>&1 &&
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > $O/gpu_suite.txt 2>&1 &&
for i in 1 2; do
  TNET_FWD_SHADOW=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/fused_fs0_$i.json 2> $O/fused_fs0_$i.err &&
  TNET_FWD_SHADOW=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/fused_fs1_$i.json 2> $O/fused_fs1_$i.err || exit 1
done &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --hip-trace --marker-trace --output-format csv -d "$R/$O/armed" -o armed \
  -- python3 "$R/tools/armed_step_trace.py" run > "$R/$O/armed_run.json" 2> "$R/$O/armed_run.err" &&
cd "$R" &&
{ python3 tools/armed_step_trace.py summarize $O/armed > $O/armed_summary.json; true; } &&
timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > $O/forcedp.json 2> $O/forcedp.err &&
TNET_DP_RESERVE_CUS=16 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > $O/forcedp_res16.json 2> $O/forcedp_res16.err &&
TNET_DP_RESERVE_CUS=16 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > $O/forcedp_res16_b.json 2> $O/forcedp_res16_b.err &&
timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline > $O/forcedp_b.json 2> $O/forcedp_b.err
rc=$?
echo "r6c rc=$rc"
exit $rc
