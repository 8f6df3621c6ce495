#!/bin/bash
# round-6 session: the driver's command x2, a 100-step run, rocprof step stats + timeline, in-step MFMA busy
set -e
out=gpurun_out/r6d7
mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver$i.txt 2>&1 || { tail -20 $out/bench_driver$i.txt; exit 1; }
  grep '"metric"' $out/bench_driver$i.txt
done
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > $out/bench100.txt 2>&1
grep -o '"ms_per_step": [0-9.]*' $out/bench100.txt
timeout -k 10 300 tools/prof_step.sh r6_final --steps 40 --warmup 10
python tools/prof_summary.py gpurun_out/prof_r6_final > $out/prof_summary.txt 2>&1 || true
python tools/prof_timeline.py gpurun_out/prof_r6_final > $out/timeline.txt 2>&1 || true
timeout -k 10 300 bash tools/pmc_step_mfma.sh
python tools/pmc_step_mfma_summary.py gpurun_out/pmc_step_mfma > $out/pmc_step_mfma.txt 2>&1 || true
tail -25 $out/pmc_step_mfma.txt
