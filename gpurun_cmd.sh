set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -q -rf -x --timeout 200 --timeout-method thread tests/test_gpu_reader.py tests/test_reader.py > gpurun_out/r3_reader_tests.txt 2>&1 &&
timeout -k 10 400 python3 -u tools/reader_bench.py 400000 > gpurun_out/r3_reader_bench.json 2> gpurun_out/r3_reader_bench.err
echo "done $?"
