set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "gather" > gpurun_out/r3s3_gather_kernel.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3s3_gpu_suite_tail.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py > gpurun_out/ab_dnn4_tail_$i.json 2>/dev/null &&
  TNET_GATHER_TAIL=0 timeout -k 10 200 python3 -u bench.py > gpurun_out/ab_dnn4_notail_$i.json 2>/dev/null &&
  timeout -k 10 200 python3 -u bench.py --config mlp3 > gpurun_out/ab_mlp3_tail_$i.json 2>/dev/null &&
  TNET_GATHER_TAIL=0 timeout -k 10 200 python3 -u bench.py --config mlp3 > gpurun_out/ab_mlp3_notail_$i.json 2>/dev/null || exit 1
done
echo "done $?"
