#!/bin/bash
# round 6, final evidence: the whole GPU suite, smoke(), the default bench line (with the CPU baseline), its kernel
# trace, the PMC passes of the roofline GEMM set, the other BASELINE configs' lines, the one-rank DP lines
set -o pipefail
R=$(pwd)
O=gpurun_out/final
mkdir -p $O
export TMPDIR=/tmp
T="timeout -k 10"
$T 1000 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.txt 2>&1 &&
$T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 &&
$T 420 python3 bench.py > $O/bench.json 2> $O/bench.err &&
$T 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_window.json 2> $O/bench_window.err &&
cd /tmp &&
$T 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_stats" -o bench --output-format csv \
  -- python3 "$R/bench.py" --no-cpu-baseline > "$R/$O/bench_prof.json" 2> "$R/$O/prof_stats.err" &&
$T 120 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/pmc_fetch" -o pmc --output-format csv \
  -- python3 "$R/tools/gemm_pmc.py" layer 20 > "$R/$O/pmc_fetch.log" 2>&1 &&
$T 120 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/pmc_write" -o pmc --output-format csv \
  -- python3 "$R/tools/gemm_pmc.py" layer 20 > "$R/$O/pmc_write.log" 2>&1 &&
cd "$R" &&
$T 300 python3 bench.py --config mlp3 > $O/mlp3.json 2> $O/mlp3.err &&
$T 300 python3 bench.py --config dnn5 --no-cpu-baseline > $O/dnn5.json 2> $O/dnn5.err &&
$T 300 python3 bench.py --force-dp --no-cpu-baseline > $O/dnn4_dp.json 2> $O/dnn4_dp.err &&
TNET_DP_RESERVE_CUS=16 $T 300 python3 bench.py --force-dp --no-cpu-baseline > $O/dnn4_dp_res16.json 2> $O/dnn4_dp_res16.err &&
$T 300 python3 bench.py --config mlp3 --force-dp --no-cpu-baseline > $O/mlp3_dp.json 2> $O/mlp3_dp.err &&
$T 300 python3 bench.py --config mlp3 --force-dp --bunch 256 --no-cpu-baseline > $O/mlp3_dp_b256.json 2> $O/mlp3_dp_b256.err &&
$T 300 python3 tools/rbm_bench.py 256 2000 10 > $O/rbm256.json 2> $O/rbm256.err &&
$T 300 python3 tools/rbm_bench.py 1024 1000 4 > $O/rbm1024.json 2> $O/rbm1024.err &&
$T 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135.json 2> $O/rnn135.err &&
$T 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000.json 2> $O/rnn4000.err
rc=$?
echo "final rc=$rc"
exit $rc
