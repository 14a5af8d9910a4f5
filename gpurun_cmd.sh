set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./tools/reduce_dpp_check > gpurun_out/r4s2_dpp.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/diag_step_resync.py > gpurun_out/r4s1_resync.txt 2>&1
timeout -k 10 900 python3 -u -m pytest -x -q -rf --timeout 400 --timeout-method thread -s \
  "tests/test_ex01.py::test_every_step_of_the_epoch_matches_reference_step" tests/test_gpu_dp.py tests/test_gpu_kernels.py -k "softmax or dp or every_step or colsum or slabs" > gpurun_out/r4s1_new_b.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r4s1_bench.json 2> gpurun_out/r4s1_bench.err &&
TNET_SOFTMAX_ROWS=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4s1_bench_sm1.json 2> gpurun_out/r4s1_bench_sm1.err &&
TNET_SOFTMAX_ROWS=4 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4s1_bench_sm4.json 2> gpurun_out/r4s1_bench_sm4.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > gpurun_out/r4s1_bench_fdp.json 2> gpurun_out/r4s1_bench_fdp.err
echo "done $?"
