set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 60 ./tools/reduce_dpp_check > $O/dpp.txt 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -v -rf --timeout 120 --timeout-method thread tests/test_gpu_rnn.py -k bptt_chain > $O/rnn_chain.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -x -v -rf --timeout 400 --timeout-method thread -s \
  "tests/test_ex01.py::test_every_step_of_the_epoch_matches_reference_step" tests/test_gpu_dp.py tests/test_gpu_recovery.py \
  tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -k "every_step or dp or failed_step or first_layer or softmax or colsum or slabs or gather" > $O/tests.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
TNET_SOFTMAX_ROWS=1 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_sm1.json 2> $O/bench_sm1.err &&
TNET_SOFTMAX_ROWS=2 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_sm2.json 2> $O/bench_sm2.err &&
TNET_SOFTMAX_ROWS=4 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_sm4.json 2> $O/bench_sm4.err &&
TNET_SOFTMAX_ROWS=1 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_sm1b.json 2> $O/bench_sm1b.err &&
TNET_SOFTMAX_ROWS=2 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_sm2b.json 2> $O/bench_sm2b.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/bench_fdp.json 2> $O/bench_fdp.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --bunch 128 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3_b128_fdp.json 2> $O/bench_mlp3_b128_fdp.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --bunch 128 --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3_b128.json 2> $O/bench_mlp3_b128.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/bench_mlp3.json 2> $O/bench_mlp3.err &&
timeout -k 10 300 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_rnn.py tests/test_gpu_fullsize.py -k "rnn or utterance or recurrent" > $O/rnn_tests.txt 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135.txt 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000.txt 2>&1 &&
TNET_RNN_BPTT_CHAIN=0 timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > $O/rnn135_nochain.txt 2>&1 &&
TNET_RNN_BPTT_CHAIN=0 timeout -k 10 300 python3 tools/rnn_bench.py 4 4000 > $O/rnn4000_nochain.txt 2>&1 &&
timeout -k 10 120 ./tools/cohab_probe steal 16 > $O/cohab_steal16.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/diag_step_resync.py > $O/resync.txt 2>&1
echo "done $?"
