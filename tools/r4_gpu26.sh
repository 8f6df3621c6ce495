#!/bin/bash
# r4 final tree re-check: the whole GPU tier + smoke
mkdir -p gpurun_out/r4zz
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4zz/gpu_tier.txt 2>&1
rc=$?
tail -3 gpurun_out/r4zz/gpu_tier.txt
grep -E "^FAILED|^ERROR" gpurun_out/r4zz/gpu_tier.txt | head
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4zz/smoke.txt 2>&1 || exit 3
tail -1 gpurun_out/r4zz/smoke.txt
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4zz/drv.json 2>>gpurun_out/r4zz/bench.log || exit 4
echo "driver cmd mlp4: $(python -c "import json;print(json.load(open('gpurun_out/r4zz/drv.json'))['ms_per_step'])")"
