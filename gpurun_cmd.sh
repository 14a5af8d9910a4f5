set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
hipcc --offload-arch=gfx950 -O3 -o tools/mfma_peak tools/mfma_peak.hip && \
timeout -k 10 120 tools/mfma_peak > gpurun_out/mfma_peak.log 2>&1 && \
timeout -k 10 600 python tools/gemm_sweep.py 20 > gpurun_out/sweep.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err
echo "done $?"
