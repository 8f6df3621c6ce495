#!/bin/bash
# r4: new fast-path tests, engine tests, then backward-order A/B (same box) + step trace
mkdir -p gpurun_out/r4c
timeout -k 10 900 python -u -m pytest tests/test_fastpaths_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4c/tests.txt 2>&1
rc=$?; tail -40 gpurun_out/r4c/tests.txt | grep -E "PASS|FAIL|Error|error|passed|failed" | tail -30
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
for o in 0 1; do
  PZ_BWD_ORDER=$o timeout -k 10 120 python bench.py --gpus 1 --steps 100 --warmup 20 > gpurun_out/r4c/mlp4_o$o.$i.json 2>>gpurun_out/r4c/bench.log || exit 3
  echo "mlp4 order=$o: $(python -c "import json;print(json.load(open('gpurun_out/r4c/mlp4_o$o.$i.json'))['ms_per_step'])")"
  PZ_BWD_ORDER=$o timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4c/f8_o$o.$i.json 2>>gpurun_out/r4c/bench.log || exit 3
  echo "mlp8192 order=$o: $(python -c "import json;print(json.load(open('gpurun_out/r4c/f8_o$o.$i.json'))['ms_per_step'])")"
done
done
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4c/drv.json 2>>gpurun_out/r4c/bench.log && cat gpurun_out/r4c/drv.json
bash tools/prof_step.sh r4_order --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_order > gpurun_out/r4c/prof_order_summary.txt 2>&1
bash tools/prof_step.sh r4_order_f8 --config mlp8192 --steps 30 --warmup 10 && python tools/prof_summary.py gpurun_out/prof_r4_order_f8 > gpurun_out/r4c/prof_order_f8_summary.txt 2>&1
tail -16 gpurun_out/r4c/prof_order_summary.txt
