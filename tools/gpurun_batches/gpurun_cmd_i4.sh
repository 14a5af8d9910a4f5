set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i4
mkdir -p $O
# CuMatrix row-stride skew (TNET_STRIDE_SKEW=1 default: +32 elements where the padded stride is a multiple of
# 1024) vs the plain rounding, interleaved: dnn4 and MLP3; then the whole GPU suite on the default
for r in 1 2; do
  TNET_STRIDE_SKEW=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/sk1_$r.json 2> $O/sk1_$r.err &&
  TNET_STRIDE_SKEW=0 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/sk0_$r.json 2> $O/sk0_$r.err || exit 1
done &&
TNET_STRIDE_SKEW=1 timeout -k 10 200 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_sk1.json 2> $O/mlp3_sk1.err &&
TNET_STRIDE_SKEW=0 timeout -k 10 200 python3 bench.py --config mlp3 --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_sk0.json 2> $O/mlp3_sk0.err &&
timeout -k 10 700 python3 -u -m pytest tests -x -q -rf -m gpu --timeout 120 --timeout-method thread > $O/gpu_suite.txt 2>&1
echo "done $?"
