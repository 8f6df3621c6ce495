#!/bin/bash
# r4: the whole GPU tier under the line tracer (GPU-tier coverage), smoke, driver-command benches,
# a forced-comm bench whose stdout must be exactly one JSON line
mkdir -p gpurun_out/r4m
PZ_COV_GPU=1 timeout -k 10 1000 python -u tools/line_coverage.py tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4m/cov.txt 2>&1
rc=$?
grep -E "passed|failed|TOTAL|engine/|functional" gpurun_out/r4m/cov.txt | cut -c1-200 | head -20
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4m/smoke.txt 2>&1 || exit 3
tail -1 gpurun_out/r4m/smoke.txt
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4m/drv.json 2>>gpurun_out/r4m/bench.log || exit 4
  echo "driver cmd mlp4: $(python -c "import json;print(json.load(open('gpurun_out/r4m/drv.json'))['ms_per_step'])")"
done
timeout -k 10 120 python bench.py --config mlp8192 --steps 20 --warmup 5 > gpurun_out/r4m/f.json 2>>gpurun_out/r4m/bench.log || exit 4
echo "driver cmd mlp8192: $(python -c "import json;print(json.load(open('gpurun_out/r4m/f.json'))['ms_per_step'])")"
PZ_FORCE_COMM=1 timeout -k 10 120 python bench.py --steps 60 --warmup 20 > gpurun_out/r4m/t.json 2>>gpurun_out/r4m/bench.log || exit 4
echo "forced comm (torch RCCL) stdout lines: $(wc -l < gpurun_out/r4m/t.json) ms: $(python -c "import json;print(json.load(open('gpurun_out/r4m/t.json'))['ms_per_step'])")"
PZ_GRAD_DTYPE=fp32 timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4m/g32.json 2>>gpurun_out/r4m/bench.log || exit 4
echo "mlp4 fp32 grads: $(python -c "import json;print(json.load(open('gpurun_out/r4m/g32.json'))['ms_per_step'])")"
timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4m/m.json 2>>gpurun_out/r4m/bench.log || exit 4
echo "mlp4 100: $(python -c "import json;print(json.load(open('gpurun_out/r4m/m.json'))['ms_per_step'])")"
