set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --config mlp3 > gpurun_out/b_mlp3.json 2> gpurun_out/b_mlp3.err &&
timeout -k 10 400 python3 bench.py --config dnn5 > gpurun_out/b_dnn5.json 2> gpurun_out/b_dnn5.err
echo "done $?"
