# MLP3 top layer row-block kernel after the label prefetch, batched LDS staging and unrolled combine: V 1 / 3
# launch-timed with phase stamps, the old split-K form, then the fused-top parity test under both variants
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5h
mkdir -p $O
for v in 1 3; do
  TNET_TOP_ROWS_V=$v timeout -k 10 120 python tools/top_rows_bench.py --stamps >> $O/top_rows_bench.jsonl 2>> $O/bench.err || exit 1
done
TNET_TOP_ROWS=0 timeout -k 10 120 python tools/top_rows_bench.py >> $O/top_rows_bench.jsonl 2>> $O/bench.err || exit 1
for v in 1 3; do
  TNET_TOP_ROWS_V=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_kernels.py -k "affine_softmax_xent or affine_fwd" > $O/pytest_v$v.log 2>&1 || exit 1
done
