#!/bin/bash
# r4: rehearse the driver's multi-GPU bench launch on one GPU (gloo, ranks sharing the card):
# torch.distributed.run with 4 ranks, and bench.py's self-launch with 8 ranks; stdout must be ONE JSON line
mkdir -p gpurun_out/r4w
PZ_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 3 --warmup 1 --batch 1024 > gpurun_out/r4w/tr4.out 2> gpurun_out/r4w/tr4.err || exit 2
echo "torchrun 4 ranks: stdout lines $(wc -l < gpurun_out/r4w/tr4.out)"; cat gpurun_out/r4w/tr4.out | cut -c1-300
PZ_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 8 --steps 3 --warmup 1 --batch 1024 > gpurun_out/r4w/self8.out 2> gpurun_out/r4w/self8.err || exit 3
echo "self-launch 8 ranks: stdout lines $(wc -l < gpurun_out/r4w/self8.out)"; cat gpurun_out/r4w/self8.out | cut -c1-300
