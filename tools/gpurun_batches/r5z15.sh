# is the MLP3 one-rank DP step host-bound? host enqueue vs completion per step (tools/host_rate.py), fused beside it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5z15
mkdir -p $O
timeout -k 10 200 python3 tools/host_rate.py --config mlp3 --force-dp --steps 640 > $O/fdp.json 2> $O/err.txt &&
timeout -k 10 200 python3 tools/host_rate.py --config mlp3 --steps 640 > $O/fused.json 2>> $O/err.txt &&
timeout -k 10 200 python3 tools/host_rate.py --config dnn4 --force-dp --steps 200 > $O/dnn4_fdp.json 2>> $O/err.txt
