# MLP3 top layer: the row-block kernel (two softmax rows a wave, sc1 half-slab hand-off) vs the split-K form, launch
# level and in the step; its parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "softmax or affine_fwd" > $O/tests.txt 2>&1 &&
for t in 1 0 1 0; do
  TNET_TOP_ROWS=$t timeout -k 10 120 python tools/top_rows_bench.py >> $O/top_rows_bench.jsonl 2>> $O/bench.err || exit 1
done &&
for t in 1 0 1 0; do
  TNET_TOP_ROWS=$t timeout -k 10 300 python bench.py --config mlp3 --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3_t$t.json 2>> $O/bench.err || exit 1
  cp $O/mlp3_t$t.json $O/mlp3_t${t}_$(date +%s%N).json
done
