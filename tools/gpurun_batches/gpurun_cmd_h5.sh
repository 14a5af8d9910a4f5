set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h5
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -rf --timeout 400 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_dp.py tests/test_gpu_steal.py \
  -k "grad_bwd_pair or grad_bias or dp or steal or update_bwd_pair" > $O/tests.txt 2>&1 &&
for v in 1 0 1 0; do
  TNET_DP_PAIR=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_p$v.json 2>> $O/fdp.err || exit 1
  cat $O/fdp_p$v.json >> $O/fdp_all.jsonl
done &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/fused.json 2> $O/fused.err &&
TNET_DP_PAIR=1 timeout -k 10 300 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_fdp.json 2> $O/mlp3_fdp.err
echo "done $?"
