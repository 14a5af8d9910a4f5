set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "colsum or gather or softmax" > gpurun_out/r3s3_rider_kernel.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3s3_gpu_suite_rider.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab_dnn4_ride_$i.json 2>/dev/null &&
  TNET_TOP_SLABS_RIDE=0 timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > gpurun_out/ab_dnn4_noride_$i.json 2>/dev/null || exit 1
done
bash tools/evidence_configs.sh
echo "done $?"
