set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/rnn_bench.py 4 135 > gpurun_out/rnn.log 2>&1 &&
timeout -k 10 300 python3 tools/rnn_bench.py 2 4000 >> gpurun_out/rnn.log 2>&1
echo "done $?"
