set -o pipefail
mkdir -p gpurun_out/prof gpurun_out/pmc
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.log 2> gpurun_out/bench.err && \
cd /tmp && export TMPDIR=/tmp && cd $R && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --kernel-timing 0 > gpurun_out/prof_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-timing 0 > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc -o write --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-timing 0 > gpurun_out/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES -d gpurun_out/pmc -o sq --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-timing 0 > gpurun_out/pmc_sq.log 2>&1
echo "done $?"
