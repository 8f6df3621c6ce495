#!/bin/bash
# round-6 session: the round's two step-level defaults against their switches, 5 interleaved rounds, mlp4
set -e
out=gpurun_out/r6d15
mkdir -p $out
ROUNDS=5 ARGS="--steps 100 --warmup 20" timeout -k 10 1000 tools/ab_bench.sh "r6=" "no_var40=PZ_GEMM_W4=0" "no_prio=PZ_MAIN_PRIO=0" "r5_like=PZ_GEMM_W4=0,PZ_MAIN_PRIO=0" > $out/ab.txt 2>&1
cat $out/ab.txt
