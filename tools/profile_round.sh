#!/bin/bash
# One GPU call that refreshes the round's measurement evidence (run via gpurun from the repo root):
#   1. bench.py default line (N=1, with the CPU baseline)                -> gpurun_out/bench.json
#   2. rocprofv3 --kernel-trace --stats of the same bench command        -> gpurun_out/prof_stats/
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE: they do not fit one pass) over the roofline kernel
#      set (tools/gemm_pmc.py layer)                                      -> gpurun_out/pmc_{fetch,write}/
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_stats" -o bench --output-format csv \
  -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/bench_prof.json" 2> "$R/gpurun_out/prof_stats.err" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o pmc --output-format csv \
  -- python3 "$R/tools/gemm_pmc.py" layer 20 > "$R/gpurun_out/pmc_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o pmc --output-format csv \
  -- python3 "$R/tools/gemm_pmc.py" layer 20 > "$R/gpurun_out/pmc_write.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES \
  -d "$R/gpurun_out/pmc_mfma" -o pmc --output-format csv \
  -- python3 "$R/tools/gemm_pmc.py" layer 300 > "$R/gpurun_out/pmc_mfma.log" 2>&1 &&
cd "$R" &&
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > gpurun_out/clock.log 2>&1
rc=$?
echo "profile_round rc=$rc"
exit $rc
