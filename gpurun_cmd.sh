set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python3 tools/intake_bench.py 400000 16384 > gpurun_out/intake.log 2>&1 &&
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/b.json 2> gpurun_out/b.err
echo "done $?"
