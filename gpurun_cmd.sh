set -o pipefail
mkdir -p gpurun_out
for v in 1 pfloop 1 pfloop; do
  TNET_DIAG_STAMP_LIB=$v timeout -k 10 120 python3 tools/gemm_clock.py 1.0 3 >> gpurun_out/pf_$v.log 2>&1 || exit 1
done
echo "done $?"
