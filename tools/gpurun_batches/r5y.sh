# the top layer's 128x256 update paired with the shadow backward below it (one launch): parity, then dnn4 A/B
# (TNET_PAIR_WIDE=1 / 0) interleaved x3
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5y
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_shadow.py \
  tests/test_gpu_train.py tests/test_gpu_fullsize.py > $O/tests.txt 2>&1 || exit 1
for r in 1 2 3; do
  for m in 1 0; do
    TNET_PAIR_WIDE=$m timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/dnn4_w${m}_$r.json 2>> $O/bench.err || exit 1
  done
done
