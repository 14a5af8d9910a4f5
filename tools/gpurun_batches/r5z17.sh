# where the dnn4 one-rank DP step's 411 us of host enqueue goes: HIP API trace (no counters) of host_rate's replay
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z17
mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-trace --stats -d $O/fdp -o run --output-format csv -- python3 tools/host_rate.py --config dnn4 --force-dp --steps 100 > $O/fdp.json 2> $O/fdp.err &&
timeout -k 10 300 rocprofv3 --hip-trace --stats -d $O/fused -o run --output-format csv -- python3 tools/host_rate.py --config dnn4 --steps 100 > $O/fused.json 2> $O/fused.err
