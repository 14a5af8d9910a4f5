set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "bwd" > gpurun_out/kt.log 2>&1
echo "done $?"
