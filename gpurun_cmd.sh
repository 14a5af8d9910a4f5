set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 20 --warmup 5 --comm host --same-device > gpurun_out/r3_bench_n2_host.json 2> gpurun_out/r3_bench_n2_host.err &&
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench_n1_torchrun.json 2> gpurun_out/r3_bench_n1_torchrun.err &&
timeout -k 10 300 python3 bench.py --force-dp --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/r3_bench_forcedp.json 2> gpurun_out/r3_bench_forcedp.err
echo "done $?"
