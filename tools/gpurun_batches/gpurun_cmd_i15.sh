set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i15
mkdir -p $O
# the step's last two updates + gather as one mixed-configuration launch (default) vs separate (TNET_UPD_MIXED=0)
timeout -k 10 400 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  -k "update_bias_gather or update_bias_pair" > $O/tests.txt 2>&1 &&
timeout -k 10 400 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_fullsize.py -m gpu > $O/tests_train.txt 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/mixed_$r.json 2> $O/mixed_$r.err &&
  TNET_UPD_MIXED=0 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/sep_$r.json 2> $O/sep_$r.err || exit 1
done
echo "done $?"
