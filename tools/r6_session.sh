#!/bin/bash
set -e
mkdir -p gpurun_out/r6c5
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -v -s --timeout 120 --timeout-method thread -k "boundary_schedules or bit_reproducible or colsum" > gpurun_out/r6c5/tests.txt 2>&1 || { grep -E "PASS|FAIL|max \|dp\|" gpurun_out/r6c5/tests.txt | cut -c1-300; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r6c5/tests.txt | cut -c1-200
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "base=" "prefetch=PZ_PREFETCH=1" "prio=PZ_FIRST_PRIO=1" "both=PZ_PREFETCH=1,PZ_FIRST_PRIO=1" > gpurun_out/r6c5/ab.txt 2>&1
cat gpurun_out/r6c5/ab.txt
PZ_PREFETCH=1 PZ_FIRST_PRIO=1 timeout -k 10 300 tools/prof_step.sh r6_both --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_both > gpurun_out/r6c5/timeline_both.txt 2>&1 || true
timeout -k 10 300 tools/prof_step.sh r6_base --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_base > gpurun_out/r6c5/timeline_base.txt 2>&1 || true
PZ_FORCE_COMM=1 PZ_COMM=proxy PZ_COMM_PROXY_WGS=16 PZ_ZERO=1 PZ_COMM_PROXY_GBPS=1e12 timeout -k 10 300 tools/prof_step.sh r6_zero_dpnone --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_zero_dpnone > gpurun_out/r6c5/timeline_zero_dpnone.txt 2>&1 || true
PZ_FORCE_COMM=1 PZ_COMM=proxy PZ_COMM_PROXY_WGS=16 PZ_COMM_PROXY_GBPS=1e12 timeout -k 10 300 tools/prof_step.sh r6_dpnone --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_dpnone > gpurun_out/r6c5/timeline_dpnone.txt 2>&1 || true
