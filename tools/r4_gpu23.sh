#!/bin/bash
# r4: schedule knobs re-checked on the r4 tree (sample prefetch placements, deferred L2 update, merge)
mkdir -p gpurun_out/r4v
for i in 1 2; do
  for env in "PZ_OPT_MERGE=1" "PZ_PREFETCH_MAIN=1" "PZ_PREFETCH=1" "PZ_OPT_DEFER=1" "PZ_OPT_MERGE=0"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4v/m.json 2>>gpurun_out/r4v/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4v/m.json'))['ms_per_step'])")"
  done
  for env in "PZ_OPT_MERGE=1" "PZ_OPT_DEFER=1" "PZ_OPT_MERGE=0"; do
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4v/f.json 2>>gpurun_out/r4v/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4v/f.json'))['ms_per_step'])")"
  done
done
