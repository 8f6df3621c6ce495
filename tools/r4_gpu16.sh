#!/bin/bash
# r4: side-stream update grid cap (PZ_OPT_SIDE_GRID) A/B
mkdir -p gpurun_out/r4p2
for i in 1 2; do
  for g in 0 1024 512 256; do
    PZ_OPT_SIDE_GRID=$g timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4p2/m.json 2>>gpurun_out/r4p2/bench.log || exit 3
    echo "mlp4 side_grid=$g: $(python -c "import json;print(json.load(open('gpurun_out/r4p2/m.json'))['ms_per_step'])")"
    PZ_OPT_SIDE_GRID=$g timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4p2/f.json 2>>gpurun_out/r4p2/bench.log || exit 3
    echo "mlp8192 side_grid=$g: $(python -c "import json;print(json.load(open('gpurun_out/r4p2/f.json'))['ms_per_step'])")"
  done
done
for i in 1 2; do
  for env in "PZ_MAIN_PRIO=0" "PZ_MAIN_PRIO=-1"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4p2/m.json 2>>gpurun_out/r4p2/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4p2/m.json'))['ms_per_step'])")"
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4p2/f.json 2>>gpurun_out/r4p2/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4p2/f.json'))['ms_per_step'])")"
  done
done
