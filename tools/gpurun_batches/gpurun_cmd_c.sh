set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v -rf --timeout 400 --timeout-method thread \
  tests/test_gpu_kernels.py -k "d4 or d8" > $O/tests_direct.txt 2>&1 &&
timeout -k 10 600 python3 -u tools/gemm_sweep.py 50 auto,m64x128d4,m64x128d8,m128x128d4,auto \
  '[["fwd",1024,2048,2048],["bwd",1024,2048,2048],["upd",1024,2048,2048],["fwd",1024,2048,4000],["upd",1024,2048,4000]]' > $O/sweep_direct.txt 2>&1 &&
timeout -k 10 900 python3 -u -m pytest -x -v -rf --timeout 400 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_dp.py tests/test_gpu_rnn.py \
  -k "grad_bias_gather or sgd or dp or update_bias_gather or bptt" > $O/tests.txt 2>&1 &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_512.json 2> $O/fdp_512.err &&
TNET_SGD_BLOCKS=256 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_256.json 2> $O/fdp_256.err &&
TNET_SGD_BLOCKS=1024 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_1024.json 2> $O/fdp_1024.err &&
TNET_SGD_BLOCKS=8192 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_8192.json 2> $O/fdp_8192.err &&
TNET_DP_APPLY_STREAM=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_noapplystream.json 2> $O/fdp_noapplystream.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --force-dp --no-cpu-baseline > $O/fdp_512b.json 2> $O/fdp_512b.err &&
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/fused.json 2> $O/fused.err
echo "done $?"
