#!/bin/bash
# round-6 session: preload depth of the one-round optimizer launches (PZ_OPT_PRE_SMALL) A/B, mlp4
set -e
out=gpurun_out/r6d13
mkdir -p $out
PZ_OPT_PRE_SMALL=4 timeout -k 10 240 python -u -m pytest tests/test_engine_gpu.py -q --timeout 120 --timeout-method thread -k "reproducible or bench_shape" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "base=" "pre2=PZ_OPT_PRE_SMALL=2" "pre4=PZ_OPT_PRE_SMALL=4" > $out/ab.txt 2>&1
cat $out/ab.txt
