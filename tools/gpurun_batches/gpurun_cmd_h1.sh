set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h1
mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1
echo "done $?"
