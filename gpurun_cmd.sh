set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -q -rf -x --timeout 300 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_kernels.py -k "pair or train or mlp3" > gpurun_out/r3_pair_tests.txt 2>&1 &&
for i in 1 2 3; do
timeout -k 10 120 python3 -u bench.py --config mlp3 --no-cpu-baseline --breakdown-steps 0 > gpurun_out/r3_mlp3_pair_$i.json 2>/dev/null &&
TNET_GEMM_PAIR=0 timeout -k 10 120 python3 -u bench.py --config mlp3 --no-cpu-baseline --breakdown-steps 0 > gpurun_out/r3_mlp3_nopair_$i.json 2>/dev/null || exit 1
done &&
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --breakdown-steps 0 > gpurun_out/r3_dnn4_after_pair.json 2>/dev/null
echo "done $?"
