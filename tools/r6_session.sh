#!/bin/bash
# round-6 session: cost of deterministic reductions on the final tree (mlp4), priority stream on fp8 mlp8192
set -e
out=gpurun_out/r6d17
mkdir -p $out
ROUNDS=3 ARGS="--steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "det=" "nondet=PZ_DETERMINISTIC=0" > $out/ab_det.txt 2>&1
cat $out/ab_det.txt
ROUNDS=3 ARGS="--config mlp8192 --steps 100 --warmup 20" timeout -k 10 900 tools/ab_bench.sh "prio=" "noprio=PZ_MAIN_PRIO=0" > $out/ab_fp8_prio.txt 2>&1
cat $out/ab_fp8_prio.txt
