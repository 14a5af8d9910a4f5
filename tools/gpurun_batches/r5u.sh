# evidence: a sustained 1000-step dnn4 line; rocprofv3 kernel-trace stats of the one-rank DP steps (dnn4, MLP3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$(pwd)
O=gpurun_out/r5u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 1000 --warmup 20 --no-cpu-baseline --breakdown-steps 0 > $O/dnn4_1000.json 2> $O/bench.err || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_fdp_dnn4" -o fdp --output-format csv \
  -- python3 "$R/bench.py" --force-dp --no-cpu-baseline --steps 100 --kernel-timing 0 --breakdown-steps 0 > "$R/$O/fdp_dnn4.json" 2>> "$R/$O/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$O/prof_fdp_mlp3" -o fdp --output-format csv \
  -- python3 "$R/bench.py" --config mlp3 --force-dp --no-cpu-baseline --steps 400 --kernel-timing 0 --breakdown-steps 0 > "$R/$O/fdp_mlp3.json" 2>> "$R/$O/bench.err"
