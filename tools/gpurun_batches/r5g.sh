# MLP3 top layer row-block kernel: B-fragment variants (TNET_TOP_ROWS_V 1/2/3) launch-timed, with phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5g
mkdir -p $O
for v in 1 2 3; do
  TNET_TOP_ROWS_V=$v timeout -k 10 120 python tools/top_rows_bench.py --stamps >> $O/top_rows_bench.jsonl 2>> $O/bench.err || exit 1
done
TNET_TOP_ROWS=0 timeout -k 10 120 python tools/top_rows_bench.py >> $O/top_rows_bench.jsonl 2>> $O/bench.err
