set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4b
mkdir -p $O
NB="--newbob --start-halving-inc 0.01 --end-halving-inc 0.001 --epochs 20"
rc=0
for s in 1 2 3; do
  timeout -k 10 400 python3 -u tools/dp_accuracy.py --corpus ex01 --worlds 1 --bunch 1024 --lr 8 $NB --seed $s \
    --progress $O/ex01_w1_s$s.jsonl > $O/ex01_w1_s$s.log 2>&1 || { rc=$?; break; }
  timeout -k 10 400 python3 -u tools/dp_accuracy.py --corpus ex01 --worlds 8 --bunch 128 --scale none --lr 8 $NB --seed $s \
    --progress $O/ex01_w8strong_s$s.jsonl > $O/ex01_w8strong_s$s.log 2>&1 || { rc=$?; break; }
  timeout -k 10 400 python3 -u tools/dp_accuracy.py --corpus teacher --worlds 1 --lr 1 --warmup 0.5 $NB --seed $s \
    --progress $O/teacher_w1_s$s.jsonl > $O/teacher_w1_s$s.log 2>&1 || { rc=$?; break; }
  timeout -k 10 400 python3 -u tools/dp_accuracy.py --corpus teacher --worlds 8 --lr 0.5 --scale linear --warmup 0.5 $NB --seed $s \
    --progress $O/teacher_w8lin4_s$s.jsonl > $O/teacher_w8lin4_s$s.log 2>&1 || { rc=$?; break; }
done
echo "done $rc"
