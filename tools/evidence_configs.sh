#!/bin/bash
# The round's secondary-configuration evidence in one GPU call (run via gpurun from the repo root),
# next to tools/profile_round.sh (the metric config):
#   bench.py --config mlp3 / dnn5 (BASELINE configs 2 and 3, with their CPU baselines) -> gpurun_out/cfg/
#   rocprofv3 kernel trace of the MLP3 step and of the bunch-256 RBM step
#   tools/rbm_bench.py at bunch 256 / 1024 (config 4), tools/rnn_bench.py at 135 / 4000 senones (config 5)
# Every GPU step has its own time limit; the chain stops at the first failure.
# tools/evidence_collect.py turns the directory into profiles/<round>_*.
set -o pipefail
R=$(pwd)
O=gpurun_out/cfg
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --config mlp3 > $O/bench_mlp3.json 2> $O/bench_mlp3.err &&
timeout -k 10 300 python3 bench.py --config dnn5 > $O/bench_dnn5.json 2> $O/bench_dnn5.err &&
timeout -k 10 300 python3 tools/rbm_bench.py 256 2000 10 > $O/rbm256.json 2>&1 &&
timeout -k 10 300 python3 tools/rbm_bench.py 1024 1000 4 > $O/rbm1024.json 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135.txt 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 2 4000 > $O/rnn4000.txt 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_mlp3" -o mlp3 --output-format csv \
  -- python3 "$R/bench.py" --config mlp3 --no-cpu-baseline --steps 300 --kernel-timing 0 \
  > "$R/$O/bench_mlp3_prof.json" 2> "$R/$O/prof_mlp3.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_rbm256" -o rbm --output-format csv \
  -- python3 "$R/tools/rbm_bench.py" 256 500 1 > "$R/$O/rbm256_prof.json" 2> "$R/$O/prof_rbm256.err"
rc=$?
echo "evidence_configs rc=$rc"
exit $rc
