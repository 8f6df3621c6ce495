#!/bin/bash
# round-6 session: 8-rank gloo rehearsal of the driver's DP bench command (all ranks on the one GPU; host
# collectives, so the time is meaningless — the check is that the 8-rank sharded-optimizer path runs and
# reports one JSON line), then the forced 1-rank RCCL bench with the sharded optimizer
set -e
out=gpurun_out/r6d14
mkdir -p $out
PZ_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29541 bench.py --gpus 8 --steps 3 --warmup 1 > $out/bench_gloo8.txt 2>&1 || { tail -30 $out/bench_gloo8.txt; exit 1; }
grep '"metric"' $out/bench_gloo8.txt | cut -c1-160
grep -o '"optimizer_sharding": "[a-z0-9]*"\|"parallelism": "[a-z0-9]*"\|"n_gpus": [0-9]*' $out/bench_gloo8.txt
PZ_FORCE_COMM=1 PZ_ZERO=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29542 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $out/bench_forced_zero.txt 2>&1 || { tail -30 $out/bench_forced_zero.txt; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"optimizer_sharding": "[a-z0-9]*"' $out/bench_forced_zero.txt
