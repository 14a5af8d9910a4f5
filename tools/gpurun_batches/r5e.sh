# the backward from the transposed weight shadow with the LDS-staged shadow stores (TNET_BWD_SHADOW 1 / 2 / 0 A/B),
# the MLP3 top layer's row-block kernel (TNET_TOP_ROWS 1 / 0 A/B), their parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shadow.py \
  tests/test_gpu_kernels.py -k "shadow or softmax or affine_fwd or transpose or bwd_colsum or update or pair" > $O/tests.txt 2>&1 &&
for m in 1 2 0 1 2 0; do
  TNET_BWD_SHADOW=$m timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/dnn4_s$m.json 2>> $O/bench.err || exit 1
  cp $O/dnn4_s$m.json $O/dnn4_s${m}_$(date +%s%N).json
done &&
for t in 1 0 1 0; do
  TNET_TOP_ROWS=$t timeout -k 10 300 python bench.py --config mlp3 --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3_t$t.json 2>> $O/bench.err || exit 1
  cp $O/mlp3_t$t.json $O/mlp3_t${t}_$(date +%s%N).json
done
