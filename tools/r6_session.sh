#!/bin/bash
# round-6 session: the paired partner's update on the compute stream at the step end (PZ_PARTNER_MAIN) A/B,
# mlp4 (bf16) and mlp8192 (fp8), + the fp8 timeline with it
set -e
out=gpurun_out/r6d9
mkdir -p $out
PZ_PARTNER_MAIN=1 timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread -k "reproducible or bench_shape" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 600 tools/ab_bench.sh "base=" "pmain=PZ_PARTNER_MAIN=1" > $out/ab_mlp4.txt 2>&1
cat $out/ab_mlp4.txt
ROUNDS=3 ARGS="--config mlp8192 --steps 100 --warmup 20" timeout -k 10 600 tools/ab_bench.sh "base=" "pmain=PZ_PARTNER_MAIN=1" > $out/ab_fp8.txt 2>&1
cat $out/ab_fp8.txt
PZ_PARTNER_MAIN=1 timeout -k 10 300 tools/prof_step.sh r6_fp8_pmain --config mlp8192 --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_fp8_pmain > $out/timeline_fp8_pmain.txt 2>&1 || true
PZ_PARTNER_MAIN=1 timeout -k 10 300 tools/prof_step.sh r6_pmain --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_pmain > $out/timeline_pmain.txt 2>&1 || true
