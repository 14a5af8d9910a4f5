set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h8
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q -rf --timeout 400 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_dp.py \
  -k "grad_pair_gather or grad_bias_gather or grad_bwd_pair or dp or update_bias_gather" > $O/tests.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_fdp.json 2> $O/mlp3_fdp.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3.json 2> $O/mlp3.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp.json 2> $O/fdp.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/fused.json 2> $O/fused.err &&
for s in 1 2 3 4 5; do
  timeout -k 10 400 python3 -u tools/dp_accuracy.py --corpus ex01 --worlds 8 --bunch 1024 --lr 0.5 --scale linear --warmup 1.0 \
    --newbob --start-halving-inc 0.01 --end-halving-inc 0.001 --epochs 20 --cv-bunch 128 --seed $s \
    --progress $O/ex01_w8weak_lr4_s$s.jsonl > $O/ex01_w8weak_lr4_s$s.log 2>&1 || exit 1
done
echo "done $?"
