#!/bin/bash
# round-6 session: per-step GPU periods of the driver's bench command (warm-up ramp)
set -e
out=gpurun_out/r6d8
mkdir -p $out
timeout -k 10 30 rocm-smi --showclocks > $out/clocks_before.txt 2>&1 || true
PZ_BENCH_SERIES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/series1.txt 2>&1
PZ_BENCH_SERIES=1 timeout -k 10 300 python bench.py --gpus 1 --steps 60 --warmup 5 > $out/series2.txt 2>&1
timeout -k 10 30 rocm-smi --showclocks > $out/clocks_after.txt 2>&1 || true
grep -h "step periods\|ms_per_step" $out/series1.txt $out/series2.txt | cut -c1-900
