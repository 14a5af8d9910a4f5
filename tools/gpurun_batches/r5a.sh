set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5a
timeout -k 10 60 ./tools/reduce_dpp_check > gpurun_out/r5a/dpp.txt 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "grad_bias_gather or softmax" tests/test_gpu_rnn.py tests/test_gpu_reader.py > gpurun_out/r5a/tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r5a/dnn4.json 2> gpurun_out/r5a/dnn4.err &&
timeout -k 10 300 python bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/r5a/mlp3.json 2> gpurun_out/r5a/mlp3.err &&
timeout -k 10 300 python bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/r5a/mlp3dp.json 2> gpurun_out/r5a/mlp3dp.err
