#!/bin/bash
set -e
mkdir -p gpurun_out/r6c9
PZ_EVENT_KIND=3 timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread -k "reproducible or bench_shape" > gpurun_out/r6c9/det.txt 2>&1 || { tail -30 gpurun_out/r6c9/det.txt; exit 1; }
tail -1 gpurun_out/r6c9/det.txt
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "k0=PZ_EVENT_KIND=0" "k3=PZ_EVENT_KIND=3" "k2=PZ_EVENT_KIND=2" > gpurun_out/r6c9/ab.txt 2>&1
cat gpurun_out/r6c9/ab.txt
PZ_EVENT_KIND=3 timeout -k 10 300 tools/prof_step.sh r6_k3 --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_k3 > gpurun_out/r6c9/timeline_k3.txt 2>&1 || true
