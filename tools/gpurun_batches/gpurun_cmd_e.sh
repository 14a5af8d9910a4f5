set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rnntrace -o trace -- python3 tools/rnn_bench.py 1 135 > $O/rnn_trace_run.txt 2>&1
echo "done $?"
