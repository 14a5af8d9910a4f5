set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -q -rf -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rbm.py tests/test_gpu_fullsize.py -k "rbm" > gpurun_out/r3_rbm_tests.txt 2>&1 &&
for i in 1 2 3; do
timeout -k 10 120 python3 -u tools/rbm_bench.py 256 500 1 > gpurun_out/r3_rbm_one_$i.txt 2>/dev/null &&
TNET_GEMM_PAIR=0 timeout -k 10 120 python3 -u tools/rbm_bench.py 256 500 1 > gpurun_out/r3_rbm_two_$i.txt 2>/dev/null || exit 1
done
echo "done $?"
