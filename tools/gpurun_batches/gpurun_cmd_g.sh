set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -k "pair or direct_form or update_bias_gather or affine" > $O/tests.txt 2>&1 &&
for v in 1 2 3 1 2 3; do
  TNET_GEMM_DIRECT=$v timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_d$v.json 2>> $O/bench.err || exit 1
  cat $O/bench_d$v.json >> $O/bench_all.jsonl
done &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rnntrace -o trace -- python3 tools/rnn_bench.py 1 135 > $O/rnn_trace_run.txt 2>&1
echo "done $?"
