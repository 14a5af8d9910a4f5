set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r4i1
mkdir -p $O
# the coalesced k-contiguous direct form (m64x128c8 / c4): bit identity to the ring, the backward paths it now
# serves, then the backward shapes and the SGD step with TNET_GEMM_KC=1 (default) / 0 interleaved
timeout -k 10 500 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -m gpu \
  -k "direct_form or c8 or c4 or bwd or pair or slabs" > $O/tests.txt 2>&1 &&
timeout -k 10 300 python3 -u tools/gemm_sweep.py 50 auto,m64x128k64s2,m64x128c4 \
  '[["bwd",1024,2048,2048],["bwdcs",1024,2048,2048],["bwd",1024,2048,4000],["fwd",1024,2048,2048]]' > $O/sweep.txt 2>&1 &&
for r in 1 2; do
  TNET_GEMM_KC=1 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/kc1_$r.json 2> $O/kc1_$r.err &&
  TNET_GEMM_KC=0 timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline > $O/kc0_$r.json 2> $O/kc0_$r.err || exit 1
done
echo "done $?"
