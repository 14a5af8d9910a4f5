#!/bin/bash
# round 6, batch af: the driver's N > 1 launch rehearsed at world 4 and 8 on the one GPU (all ranks on device 0,
# gradients summed through host memory): rendezvous, the shard ranges, the reduction check, max-over-ranks timing and
# teardown at the rank counts the driver's scaling run uses
set -o pipefail
O=gpurun_out/r6af
mkdir -p $O
export TMPDIR=/tmp OMP_NUM_THREADS=2
T="timeout -k 10"
for N in 4 8; do
  P=$((29500 + N))
  $T 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $P \
    bench.py --gpus $N --steps 3 --warmup 1 --no-cpu-baseline --cache 4096 --comm host --same-device \
    --kernel-timing 0 --breakdown-steps 0 > $O/world$N.json 2> $O/world$N.err || exit 1
done
rc=$?
echo "r6af rc=$rc"
exit $rc
