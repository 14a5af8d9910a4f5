set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/kt.log 2>&1 &&
timeout -k 10 900 python3 tools/gemm_sweep.py 30 m64x128k64s2,m128x128k64s2,m64x128k64s3p,m64x128k64s2w42,m64x128k64s3w42p,m128x128k32s3p,m128x128k32s4p,m64x64k32s4w41 > gpurun_out/sweep.log 2>&1 &&
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 200 > gpurun_out/b.json 2>&1
echo "done $?"
