set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rnn.py tests/test_gpu_dropin.py > gpurun_out/t_rnn.log 2>&1 &&
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "update_row or softmax" >> gpurun_out/t_rnn.log 2>&1 &&
timeout -k 10 300 python3 -u tools/rnn_bench.py 4 135 > gpurun_out/rnn_bench.log 2>&1 &&
timeout -k 10 300 python3 -u tools/rnn_bench.py 2 4000 >> gpurun_out/rnn_bench.log 2>&1
echo "done $?"
