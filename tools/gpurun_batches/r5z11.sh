# the GEMM clock stamps again (r5z10's forward stamps read one workgroup's start as unwritten), twice
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z11
mkdir -p $O
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock_1.log 2>&1 &&
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock_2.log 2>&1
