set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4h7
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -rf --timeout 400 --timeout-method thread > $O/gpu_suite.txt 2>&1 &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 &&
for v in 1 0 1 0; do
  TNET_DP_PAIR=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_p$v.json 2>> $O/fdp.err || exit 1
  cat $O/fdp_p$v.json >> $O/fdp_all.jsonl
done &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/fused.json 2> $O/fused.err &&
timeout -k 10 300 python3 bench.py --config mlp3 --force-dp --steps 200 --warmup 50 --no-cpu-baseline > $O/mlp3_fdp.json 2> $O/mlp3_fdp.err &&
timeout -k 10 200 python3 tools/gemm_clock.py 1.5 5 > $O/clock.log 2>&1
echo "done $?"
