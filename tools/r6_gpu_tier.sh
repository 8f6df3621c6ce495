#!/bin/bash
# full GPU test tier (one pytest process) + smoke, as the driver runs them at round end, then a 2-rank
# gloo rehearsal of the bench's data-parallel path (both ranks on the one GPU; sharded optimizer on)
set -e
out=gpurun_out/r6tier2
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/tests.txt 2>&1 || { tail -40 $out/tests.txt; exit 1; }
tail -3 $out/tests.txt
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
PZ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $out/bench_gloo2.txt 2>&1 || { tail -30 $out/bench_gloo2.txt; exit 1; }
grep '"metric"' $out/bench_gloo2.txt | cut -c1-200
grep -o '"optimizer_sharding": "[a-z0-9]*"' $out/bench_gloo2.txt
