set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 400 --timeout-method thread tests/test_gpu_steal.py tests/test_gpu_dp.py > $O/tests.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 400 --timeout-method thread tests/test_gpu_kernels.py -k "m128x256a2 or direct_form" > $O/tests_a2.txt 2>&1 &&
for v in 1 4 1 4; do
  TNET_GEMM_DIRECT=$v timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_d$v.json 2>> $O/bench_dv.err || exit 1
  cat $O/bench_d$v.json >> $O/bench_dv.jsonl
done &&
timeout -k 10 120 ./tools/cohab_probe steal 16 > $O/cohab_steal16.txt 2>&1 &&
bash tools/profile_round.sh > $O/profile_round.log 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/bench_fdp.json 2> $O/bench_fdp.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_fused.json 2> $O/bench_fused.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/bench_fdp2.json 2> $O/bench_fdp2.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3_fdp.json 2> $O/bench_mlp3_fdp.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3.json 2> $O/bench_mlp3.err &&
timeout -k 10 300 python3 bench.py --config dnn5 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_dnn5.json 2> $O/bench_dnn5.err &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135.txt 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000.txt 2>&1
echo "done $?"
