#!/bin/bash
# r4: pair + fp8 2-WG kernel tests, fast paths, step A/B (PZ_DW_PAIR, PZ_F8_2WG, PZ_FP8_WFUSE), profiles
mkdir -p gpurun_out/r4g
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -v --timeout 300 --timeout-method thread -k "pair or split_k or fp8" > gpurun_out/r4g/ktests.txt 2>&1
grep -E "PASS|FAIL|Error" gpurun_out/r4g/ktests.txt | cut -c1-160 | tail -30
grep -q FAILED gpurun_out/r4g/ktests.txt && exit 1
timeout -k 10 600 python -u -m pytest tests/test_fastpaths_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4g/tests.txt 2>&1
grep -E "PASS|FAIL|Assertion" gpurun_out/r4g/tests.txt | cut -c1-300 | tail -14
for i in 1 2; do
for pr in 0 1; do
  PZ_DW_PAIR=$pr timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4g/m.json 2>>gpurun_out/r4g/bench.log || exit 3
  echo "mlp4 pair=$pr: $(python -c "import json;print(json.load(open('gpurun_out/r4g/m.json'))['ms_per_step'])")"
done
for cfg in "0 0 0" "1 0 0" "1 1 0" "1 1 1"; do
  set -- $cfg
  PZ_DW_PAIR=$1 PZ_F8_2WG=$2 PZ_FP8_WFUSE=$3 timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4g/f8.json 2>>gpurun_out/r4g/bench.log || exit 3
  echo "mlp8192 pair=$1 2wg=$2 wfuse=$3: $(python -c "import json;print(json.load(open('gpurun_out/r4g/f8.json'))['ms_per_step'])")"
done
done
bash tools/prof_step.sh r4_pair --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_pair > gpurun_out/r4g/prof_pair.txt 2>&1
bash tools/prof_step.sh r4_f8 --config mlp8192 --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_f8 > gpurun_out/r4g/prof_f8.txt 2>&1
tail -13 gpurun_out/r4g/prof_pair.txt | cut -c1-130
tail -11 gpurun_out/r4g/prof_f8.txt | cut -c1-130
