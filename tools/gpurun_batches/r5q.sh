# the 64x64 direct-form configuration (m64x64a4) on MLP3's shapes, the affine_softmax_xent combine with its slices'
# loads batched, and the parity tests of both
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5q
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "gemm or softmax" > $O/tests.txt 2>&1 || exit 1
timeout -k 10 400 python3 tools/gemm_sweep.py 50 auto,m64x64a4,m64x64k32s4w41 \
  '[["fwd",1024,598,1024],["updb",1024,598,1024],["fwd",1024,1024,135],["fwd",1024,440,2048],["updb",1024,440,2048],["fwd",256,440,2048],["updb",256,440,2048]]' > $O/sweep.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/top_rows_bench.py > $O/top.json 2>> $O/err.txt || exit 1
timeout -k 10 200 python3 bench.py --config mlp3 --steps 400 --warmup 50 --no-cpu-baseline > $O/mlp3.json 2>> $O/err.txt
