set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -k "direct_form or a4 or a8 or d4 or d8" > $O/tests_direct.txt 2>&1 &&
TNET_GEMM_DIRECT=1 timeout -k 10 900 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -k "not a4 and not a8 and not d4 and not d8" > $O/tests_direct_on.txt 2>&1 &&
timeout -k 10 600 python3 -u tools/gemm_sweep.py 50 auto,m64x128a4,m64x128a8,m128x128a4,m64x128d4,m128x128d4,auto \
  '[["fwd",1024,2048,2048],["upd",1024,2048,2048],["fwd",1024,2048,4000],["upd",1024,2048,4000],["fwd",1024,440,2048]]' > $O/sweep_direct.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_ring.json 2> $O/bench_ring.err &&
TNET_GEMM_DIRECT=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_direct.json 2> $O/bench_direct.err &&
timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_ring100.json 2> $O/bench_ring100.err &&
TNET_GEMM_DIRECT=1 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_direct100.json 2> $O/bench_direct100.err &&
TNET_GEMM_DIRECT=1 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_direct.json 2> $O/fdp_direct.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_ring.json 2> $O/fdp_ring.err
echo "done $?"
