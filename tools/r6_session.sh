#!/bin/bash
# round-6 session: early side update A/B (PZ_UPDATE_EARLY) on the VAR 40 build + step timelines
set -e
out=gpurun_out/r6d1
mkdir -p $out
PZ_UPDATE_EARLY=1 timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread -k "reproducible or bench_shape" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "base=" "early=PZ_UPDATE_EARLY=1" > $out/ab.txt 2>&1
cat $out/ab.txt
timeout -k 10 300 tools/prof_step.sh r6_base --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_base > $out/timeline_base.txt 2>&1 || true
PZ_UPDATE_EARLY=1 timeout -k 10 300 tools/prof_step.sh r6_early --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_early > $out/timeline_early.txt 2>&1 || true
