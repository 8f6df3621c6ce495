#!/bin/bash
# r4: serial optimizer schedule (PZ_OPT_OVERLAP=0) and backward order (PZ_BWD_ORDER=1) vs default
mkdir -p gpurun_out/r4n
PZ_OPT_SERIAL=1 timeout -k 10 600 python -u -m pytest tests/test_fastpaths_gpu.py tests/test_engine_gpu.py -v --timeout 300 --timeout-method thread -k "matches_fp32_torch or fp8_natural or graph_replay or fp8_training or paired or reference" > gpurun_out/r4n/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " gpurun_out/r4n/tests.txt | cut -c1-200 | tail -30
[ $rc -le 1 ] || exit 2
for i in 1 2; do
  for env in "PZ_OPT_OVERLAP=1" "PZ_OPT_SERIAL=1" "PZ_OPT_OVERLAP=0" "PZ_BWD_ORDER=1"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4n/m.json 2>>gpurun_out/r4n/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4n/m.json'))['ms_per_step'])")"
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4n/f.json 2>>gpurun_out/r4n/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4n/f.json'))['ms_per_step'])")"
  done
done
PZ_OPT_SERIAL=1 bash tools/prof_step.sh r4_serial --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_serial > gpurun_out/r4n/tl_serial.txt 2>&1
tail -24 gpurun_out/r4n/tl_serial.txt
PZ_COV_GPU=1 PZ_LINECOV_MISSING=1 timeout -k 10 900 python -u tools/line_coverage.py tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4n/cov.txt 2>&1
echo "cov rc=$?"; grep -E "passed|failed|TOTAL" gpurun_out/r4n/cov.txt | head -3
