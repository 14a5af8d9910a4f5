# (1) the persistent-RNN hand-off probe (the XCD-local floor), (2) the MLP3 one-rank DP step at
# every bunch with the round-5 exchange schedule (r5d.sh bench, into gpurun_out/r5m)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 60 ./tools/xcd_handoff_probe > $O/xcd_handoff_probe.jsonl 2> $O/xcd_handoff_probe.err || exit 1
B="--no-cpu-baseline --breakdown-steps 0"
for b in 128 256 512 1024; do
  timeout -k 10 200 python3 bench.py --config mlp3 --bunch $b --force-dp --steps 400 --warmup 50 $B > $O/mlp3_fdp_b$b.json 2>> $O/bench.err || exit 1
  timeout -k 10 200 python3 bench.py --config mlp3 --bunch $b --steps 400 --warmup 50 $B > $O/mlp3_b$b.json 2>> $O/bench.err || exit 1
done
