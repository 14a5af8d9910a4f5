set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/doff_*.log
for v in 1 dmaoff6 dmaoff14 1 dmaoff6 dmaoff14; do
  TNET_DIAG_STAMP_LIB=$v timeout -k 10 120 python3 tools/gemm_clock.py 1.0 3 >> gpurun_out/doff_$v.log 2>&1 || exit 1
done
echo "done $?"
