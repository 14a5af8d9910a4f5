set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rnn.py tests/test_gpu_dropin.py > gpurun_out/t_rnn.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "gemv or softmax or rowvec" >> gpurun_out/t_rnn.log 2>&1 &&
timeout -k 10 300 python3 -u tools/rnn_bench.py 4 135 > gpurun_out/rnn_bench.log 2>&1 &&
timeout -k 10 300 python3 -u tools/rnn_bench.py 2 4000 >> gpurun_out/rnn_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rnn4000b -o rnn -- python3 -u tools/rnn_bench.py 2 4000 > gpurun_out/prof_rnn.log 2>&1
echo "done $?"
