set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2> gpurun_out/bench.err
echo "done $?"
