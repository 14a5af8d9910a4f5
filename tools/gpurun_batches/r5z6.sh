# the narrow top layer's K slices from the row-block kernel + the existing combine launches (TNET_TOP_SPLIT): parity,
# launch timing, MLP3 A/B interleaved x3 (fused and one-rank DP)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_train.py tests/test_ex01.py tests/test_gpu_dp.py > $O/tests.txt 2>&1 || exit 1
for m in 1 0; do
  TNET_TOP_SPLIT=$m timeout -k 10 120 python3 tools/top_rows_bench.py >> $O/top.jsonl 2>> $O/err.txt || exit 1
done
for r in 1 2 3; do
  for m in 1 0; do
    TNET_TOP_SPLIT=$m timeout -k 10 200 python3 bench.py --config mlp3 --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3_t${m}_$r.json 2>> $O/err.txt || exit 1
  done
done
for m in 1 0; do
  TNET_TOP_SPLIT=$m timeout -k 10 200 python3 bench.py --config mlp3 --force-dp --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3fdp_t${m}.json 2>> $O/err.txt || exit 1
done
