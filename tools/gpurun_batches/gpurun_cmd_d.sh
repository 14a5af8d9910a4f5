set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v -rf --timeout 300 --timeout-method thread \
  tests/test_gpu_kernels.py -k "direct_form or a4 or a8" > $O/tests_direct.txt 2>&1 &&
timeout -k 10 600 python3 -u tools/gemm_sweep.py 50 auto,m64x128a4,m64x128a8,m128x128a4,m64x128d4,m128x128d4,auto \
  '[["fwd",1024,2048,2048],["bwd",1024,2048,2048],["upd",1024,2048,2048],["fwd",1024,2048,4096],["upd",1024,2048,4096]]' > $O/sweep_direct.txt 2>&1
echo "done $?"
