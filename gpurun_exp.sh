set -o pipefail
mkdir -p gpurun_out/exp1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_kernels.py -k "softmax or train or overlap or intake" > gpurun_out/exp1/t.log 2>&1 &&
for o in 0 1 0 1; do TNET_OVERLAP_UPDATE=$o timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/exp1/b50_$o.json 2>/dev/null || exit 1; done &&
for o in 0 1; do TNET_OVERLAP_UPDATE=$o timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/exp1/b20_$o.json 2>/dev/null || exit 1; done &&
for o in 0 1; do TNET_OVERLAP_UPDATE=$o timeout -k 10 120 python3 -u bench.py --no-cpu-baseline --steps 200 --warmup 10 --config dnn5 > gpurun_out/exp1/b5_$o.json 2>/dev/null || exit 1; done
echo done $?
