set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench.py tests/test_gpu_dp.py tests/test_gpu_rnn.py tests/test_gpu_reader.py > gpurun_out/r5b/tests.txt 2>&1
