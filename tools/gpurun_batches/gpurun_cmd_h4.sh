set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=gpurun_out/r4h4
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/bench_fdp.json 2> $O/bench_fdp.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_fused.json 2> $O/bench_fused.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/bench_fdp2.json 2> $O/bench_fdp2.err &&
timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_fused100.json 2> $O/bench_fused100.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3_fdp.json 2> $O/bench_mlp3_fdp.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3.json 2> $O/bench_mlp3.err &&
timeout -k 10 300 python3 bench.py --config dnn5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_dnn5.json 2> $O/bench_dnn5.err &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135.txt 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000.txt 2>&1 &&
cd /tmp &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/pmc_write" -o pmc --output-format csv \
  -- python3 "$R/tools/gemm_pmc.py" layer 20 > "$R/$O/pmc_write.log" 2>&1
echo "done $?"
