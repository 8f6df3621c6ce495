#!/bin/bash
mkdir -p gpurun_out/r4e
timeout -k 10 600 python -u -m pytest tests/test_fastpaths_gpu.py -v --timeout 300 --timeout-method thread -k "fp8" > gpurun_out/r4e/tests.txt 2>&1
grep -E "PASS|FAIL|Assertion" gpurun_out/r4e/tests.txt | cut -c1-300 | tail -12
for i in 1 2; do
for cfg in "0 0" "0 1" "1 1"; do
  set -- $cfg
  PZ_BWD_ORDER=$1 PZ_FP8_WFUSE=$2 timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4e/f8.json 2>>gpurun_out/r4e/bench.log || exit 3
  echo "mlp8192 order=$1 wfuse=$2: $(python -c "import json;print(json.load(open('gpurun_out/r4e/f8.json'))['ms_per_step'])")"
done
done
PZ_BWD_ORDER=0 bash tools/prof_step.sh r4_f8_pad --config mlp8192 --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_f8_pad > gpurun_out/r4e/prof_f8_pad.txt 2>&1
tail -12 gpurun_out/r4e/prof_f8_pad.txt | cut -c1-150
