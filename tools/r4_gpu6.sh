#!/bin/bash
# r4: pair kernel tests + fast paths + A/B of PZ_DW_PAIR / PZ_FP8_WFUSE on the step
mkdir -p gpurun_out/r4f
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -v --timeout 300 --timeout-method thread -k "pair or split_k or weight_gradient" > gpurun_out/r4f/ktests.txt 2>&1
grep -E "PASS|FAIL|Error" gpurun_out/r4f/ktests.txt | cut -c1-200 | tail -14
grep -q FAILED gpurun_out/r4f/ktests.txt && exit 1
timeout -k 10 600 python -u -m pytest tests/test_fastpaths_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4f/tests.txt 2>&1
grep -E "PASS|FAIL|Assertion" gpurun_out/r4f/tests.txt | cut -c1-300 | tail -14
for i in 1 2; do
for pr in 0 1; do
  PZ_DW_PAIR=$pr timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4f/m.json 2>>gpurun_out/r4f/bench.log || exit 3
  echo "mlp4 pair=$pr: $(python -c "import json;print(json.load(open('gpurun_out/r4f/m.json'))['ms_per_step'])")"
  for w in 0 1; do
    PZ_DW_PAIR=$pr PZ_FP8_WFUSE=$w timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4f/f8.json 2>>gpurun_out/r4f/bench.log || exit 3
    echo "mlp8192 pair=$pr wfuse=$w: $(python -c "import json;print(json.load(open('gpurun_out/r4f/f8.json'))['ms_per_step'])")"
  done
done
done
bash tools/prof_step.sh r4_pair --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_pair > gpurun_out/r4f/prof_pair.txt 2>&1
bash tools/prof_step.sh r4_pair_f8 --config mlp8192 --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_pair_f8 > gpurun_out/r4f/prof_pair_f8.txt 2>&1
tail -13 gpurun_out/r4f/prof_pair.txt | cut -c1-130
tail -11 gpurun_out/r4f/prof_pair_f8.txt | cut -c1-130
