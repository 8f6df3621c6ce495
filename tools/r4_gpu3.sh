#!/bin/bash
mkdir -p gpurun_out/r4d
timeout -k 10 600 python -u -m pytest tests/test_fastpaths_gpu.py -v --timeout 300 --timeout-method thread -k "fp8_natural" > gpurun_out/r4d/tests.txt 2>&1
grep -E "PASS|FAIL|Assertion" gpurun_out/r4d/tests.txt | cut -c1-400 | tail -12
for i in 1 2; do
for w in 0 1; do
  PZ_BWD_ORDER=0 PZ_FP8_WFUSE=$w timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4d/f8_w$w.$i.json 2>>gpurun_out/r4d/bench.log || exit 3
  echo "mlp8192 order0 wfuse=$w: $(python -c "import json;print(json.load(open('gpurun_out/r4d/f8_w$w.$i.json'))['ms_per_step'])")"
done
done
PZ_BWD_ORDER=0 bash tools/prof_step.sh r4_f8_o0 --config mlp8192 --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_f8_o0 > gpurun_out/r4d/prof_f8_o0.txt 2>&1
PZ_BWD_ORDER=0 PZ_FP8_WFUSE=0 bash tools/prof_step.sh r4_f8_o0w0 --config mlp8192 --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_f8_o0w0 > gpurun_out/r4d/prof_f8_o0w0.txt 2>&1
tail -14 gpurun_out/r4d/prof_f8_o0.txt | cut -c1-150
tail -14 gpurun_out/r4d/prof_f8_o0w0.txt | cut -c1-150
