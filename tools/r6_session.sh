#!/bin/bash
# round-6 session: compute stream at priority -1 (PZ_MAIN_PRIO) A/B + step timeline
set -e
out=gpurun_out/r6d2
mkdir -p $out
PZ_MAIN_PRIO=1 timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread -k "reproducible or bench_shape" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "base=" "prio=PZ_MAIN_PRIO=1" > $out/ab.txt 2>&1
cat $out/ab.txt
PZ_MAIN_PRIO=1 timeout -k 10 300 tools/prof_step.sh r6_prio --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_prio > $out/timeline_prio.txt 2>&1 || true
