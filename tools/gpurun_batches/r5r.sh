# the first layer's update in the 64x64 direct form (standalone and inside the mixed last launch): parity tests, then
# dnn4 A/B (TNET_UPD64_DIRECT=0 / 1) interleaved
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_train.py tests/test_gpu_fullsize.py tests/test_gpu_shadow.py > $O/tests.txt 2>&1 || exit 1
for r in 1 2 3; do
  for m in 1 0; do
    TNET_UPD64_DIRECT=$m timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/dnn4_d${m}_$r.json 2>> $O/bench.err || exit 1
  done
done
