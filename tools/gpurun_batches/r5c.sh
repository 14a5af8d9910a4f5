set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5c
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shadow.py > gpurun_out/r5c/shadow.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r5c/dnn4.json 2> gpurun_out/r5c/dnn4.err &&
TNET_BWD_SHADOW=0 timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r5c/dnn4_nt.json 2> gpurun_out/r5c/dnn4_nt.err &&
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r5c/dnn4_b.json 2> gpurun_out/r5c/dnn4_b.err &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_ex01.py tests/test_gpu_kernels.py tests/test_gpu_bench.py tests/test_gpu_dp.py > gpurun_out/r5c/tests.txt 2>&1
