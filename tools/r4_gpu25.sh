#!/bin/bash
# r4: the paired partner's update queued behind the first-layer launch's event (PZ_SIDE_TAIL) A/B
mkdir -p gpurun_out/r4x
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_fastpaths_gpu.py -q --timeout 300 --timeout-method thread -k "paired or graph or matches_fp32_torch or reference" > gpurun_out/r4x/tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r4x/tests.txt; [ $rc -le 1 ] || exit 2
for i in 1 2 3; do
  for t in 1 0; do
    PZ_SIDE_TAIL=$t timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4x/m.json 2>>gpurun_out/r4x/bench.log || exit 3
    echo "mlp4 PZ_SIDE_TAIL=$t: $(python -c "import json;print(json.load(open('gpurun_out/r4x/m.json'))['ms_per_step'])")"
  done
done
for t in 1 0; do
  PZ_SIDE_TAIL=$t timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4x/d.json 2>>gpurun_out/r4x/bench.log || exit 3
  echo "mlp4 driver PZ_SIDE_TAIL=$t: $(python -c "import json;print(json.load(open('gpurun_out/r4x/d.json'))['ms_per_step'])")"
done
timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4x/f.json 2>>gpurun_out/r4x/bench.log || exit 3
echo "mlp8192: $(python -c "import json;print(json.load(open('gpurun_out/r4x/f.json'))['ms_per_step'])")"
bash tools/prof_step.sh r4_tail --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_tail > gpurun_out/r4x/tl.txt 2>&1
tail -12 gpurun_out/r4x/tl.txt
