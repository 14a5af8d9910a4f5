set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_frontend.py tests/test_gpu_dropin.py tests/test_gpu_train.py -x -q > gpurun_out/gpu_tests.log 2>&1
echo "done $?"
