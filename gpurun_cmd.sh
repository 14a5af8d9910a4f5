set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_rbm.py > gpurun_out/r3s3_rbm_tests.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3s3_gpu_suite_rbmtail.txt 2>&1 &&
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/rbm_bench.py 256 500 > gpurun_out/ab_rbm256_tail_$i.txt 2>&1 &&
  TNET_GATHER_TAIL=0 timeout -k 10 200 python3 -u tools/rbm_bench.py 256 500 > gpurun_out/ab_rbm256_notail_$i.txt 2>&1 &&
  timeout -k 10 200 python3 -u tools/rbm_bench.py 1024 300 > gpurun_out/ab_rbm1024_tail_$i.txt 2>&1 &&
  TNET_GATHER_TAIL=0 timeout -k 10 200 python3 -u tools/rbm_bench.py 1024 300 > gpurun_out/ab_rbm1024_notail_$i.txt 2>&1 || exit 1
done
echo "done $?"
