#!/bin/bash
# round-6 A/B of the step-boundary schedules (same box, interleaved), then a kernel-trace timeline of the best
set -e
mkdir -p gpurun_out/r6c4
timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "boundary_schedules" > gpurun_out/r6c4/tests.txt 2>&1 || { tail -30 gpurun_out/r6c4/tests.txt; exit 1; }
tail -2 gpurun_out/r6c4/tests.txt
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "base=" "prefetch=PZ_PREFETCH=1" "prio=PZ_FIRST_PRIO=1" "both=PZ_PREFETCH=1,PZ_FIRST_PRIO=1" > gpurun_out/r6c4/ab.txt 2>&1
cat gpurun_out/r6c4/ab.txt
PZ_PREFETCH=1 PZ_FIRST_PRIO=1 timeout -k 10 300 tools/prof_step.sh r6_both --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_both > gpurun_out/r6c4/timeline_both.txt 2>&1 || true
timeout -k 10 300 tools/prof_step.sh r6_base --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_base > gpurun_out/r6c4/timeline_base.txt 2>&1 || true
