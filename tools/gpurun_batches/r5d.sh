# the middle points of data parallelism on examples/01's MLP3 -- N = 8 ranks (processes on one
# GPU over the host transport, the RCCL path's exchange protocol) at 256 and 512 rows per rank (global bunch 2048 /
# 4096), 5 seeds, newbob, two learning-rate rules (linear in the global bunch with a half-epoch warm-up; half of it);
# and the one-rank data-parallel MLP3 step time at every bunch (the throughput side).
# usage: bash tools/gpurun_batches/r5d.sh bench|256|512 [rules]   (one gpurun call each: the whole set outlasts one
# call; rules default "lin half"; "n1" = the N = 1 recipe's lr 8 unscaled, "n1half" = lr 4)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5d
mkdir -p $O
if [ "$1" = bench ]; then
  for b in 128 256 512 1024; do
    timeout -k 10 300 python3 bench.py --config mlp3 --bunch $b --force-dp --steps 400 --warmup 50 --no-cpu-baseline \
      --breakdown-steps 0 > $O/mlp3_fdp_b$b.json 2> $O/mlp3_fdp_b$b.err || exit 1
    timeout -k 10 300 python3 bench.py --config mlp3 --bunch $b --steps 400 --warmup 50 --no-cpu-baseline \
      --breakdown-steps 0 > $O/mlp3_b$b.json 2> $O/mlp3_b$b.err || exit 1
  done
  exit 0
fi
b=$1
rules=${2:-lin half}
for rule in $rules; do
  if [ $b = 256 ]; then lr=2; else lr=4; fi
  if [ $rule = half ]; then lr=$(python3 -c "print($lr/2)"); fi
  if [ $rule = n1 ]; then lr=1; fi          # x 8 ranks (--scale linear) = 8, the N = 1 recipe's lr
  if [ $rule = n1half ]; then lr=0.5; fi
  for s in 1 2 3 4 5; do
    timeout -k 10 300 python3 -u tools/dp_accuracy.py --corpus ex01 --worlds 8 --bunch $b --lr $lr --scale linear \
      --warmup 0.5 --newbob --start-halving-inc 0.01 --end-halving-inc 0.001 --epochs 20 --cv-bunch 128 --seed $s \
      --progress $O/ex01_w8_b${b}_${rule}_s$s.jsonl > $O/ex01_w8_b${b}_${rule}_s$s.log 2>&1 || exit 1
  done
done
echo "done $?"
