set -o pipefail
mkdir -p gpurun_out
TNET_BENCH_TORCH_FIRST=1 timeout -k 10 300 python3 bench.py --force-dp --no-cpu-baseline --steps 30 > gpurun_out/b_dpt.json 2> gpurun_out/b_dpt.err
echo "done $?"
