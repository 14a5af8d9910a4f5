set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-timing 0 > gpurun_out/prof_bench.log 2>&1
echo "done $?"
