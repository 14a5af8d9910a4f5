set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python3 -u tools/dp_accuracy.py --corpus ex01 --worlds 8 --epochs 15 --lr 1 --bunch 128 --cache 8192 --newbob --start-halving-inc 0.01 --end-halving-inc 0.001 > gpurun_out/r3_dpacc_ex01_w8_strong.log 2>&1 &&
timeout -k 10 500 python3 -u tools/dp_accuracy.py --corpus ex01 --worlds 1 --epochs 15 --lr 8 --bunch 1024 --cache 16384 --newbob --start-halving-inc 0.01 --end-halving-inc 0.001 > gpurun_out/r3_dpacc_ex01_w1_nowarm.log 2>&1
echo "done $?"
