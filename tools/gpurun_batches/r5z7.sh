# the wide-row softmax-xent with the label loaded first and the label column's probability taken from registers
# (no dependent logit re-read at the end): softmax parity, dnn4 bench A/B interleaved x3 against the previous
# kernel (lib/libtnet_amd_smold.so, TNET_LIB_VARIANT=smold), rocprofv3 kernel stats of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z7
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  tests/test_gpu_train.py tests/test_ex01.py -k "softmax or xent or objective or step or epoch" > $O/tests.txt 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/new_$r.json 2>> $O/err.txt || exit 1
  TNET_LIB_VARIANT=smold timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/old_$r.json 2>> $O/err.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_new -o run -- python3 bench.py --no-cpu-baseline --kernel-timing 0 --breakdown-steps 0 > $O/prof_new.log 2>&1 || exit 1
TNET_LIB_VARIANT=smold timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_old -o run -- python3 bench.py --no-cpu-baseline --kernel-timing 0 --breakdown-steps 0 > $O/prof_old.log 2>&1 || exit 1
