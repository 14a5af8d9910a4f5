set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_dropin.py -x -q > gpurun_out/gpu_tests.log 2>&1
echo "done $?"
