#!/bin/bash
# round-6 session: fused fp8 VAR 42 / 43 (column sums in their own LDS region, grouped store pass) — tests + A/B
set -e
out=gpurun_out/r6d12
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fastpaths_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8 or w4 or layouts or bitmask" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
ROUNDS=3 ARGS="--config mlp8192 --steps 100 --warmup 20" timeout -k 10 600 tools/ab_bench.sh "w4=" "now4=PZ_GEMM_W4=0" > $out/ab_fp8.txt 2>&1
cat $out/ab_fp8.txt
ROUNDS=2 ARGS="--steps 100 --warmup 20" timeout -k 10 600 tools/ab_bench.sh "w4=" "now4=PZ_GEMM_W4=0" > $out/ab_mlp4.txt 2>&1
cat $out/ab_mlp4.txt
timeout -k 10 300 tools/prof_step.sh r6_fp8_w4b --config mlp8192 --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_r6_fp8_w4b > $out/timeline_fp8.txt 2>&1 || true
grep "gemm" $out/timeline_fp8.txt | head -8
