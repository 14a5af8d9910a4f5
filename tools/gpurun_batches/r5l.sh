# inline exchange with the two applies merged (MLP3), DP tests; dnn4 force-dp kernel trace (the remaining gap)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5l
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dp.py \
  tests/test_gpu_bench.py > $O/tests.txt 2>&1 || exit 1
B="--no-cpu-baseline --breakdown-steps 0"
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 400 --warmup 50 $B > $O/mlp3_fdp_$r.json 2>> $O/bench.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_dnn4_fdp -o run -- python3 bench.py --force-dp \
  --steps 30 --warmup 10 $B > $O/dnn4_fdp_trace.json 2>> $O/bench.err
