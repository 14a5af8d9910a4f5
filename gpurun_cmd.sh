set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/diag_ex01_nb.py > gpurun_out/r3_diag_nb.log 2>&1
echo "done $?"
