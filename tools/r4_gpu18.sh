#!/bin/bash
# r4 final tree: the whole GPU tier, smoke, driver-command benches, final step profiles
mkdir -p gpurun_out/r4z
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4z/gpu_tier.txt 2>&1
rc=$?
tail -3 gpurun_out/r4z/gpu_tier.txt
[ $rc -le 1 ] || exit 2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4z/smoke.txt 2>&1 || exit 3
tail -1 gpurun_out/r4z/smoke.txt
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4z/drv$i.json 2>>gpurun_out/r4z/bench.log || exit 4
  echo "driver cmd mlp4: $(python -c "import json;print(json.load(open('gpurun_out/r4z/drv$i.json'))['ms_per_step'])")"
done
timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4z/m.json 2>>gpurun_out/r4z/bench.log || exit 4
echo "mlp4 100: $(python -c "import json;print(json.load(open('gpurun_out/r4z/m.json'))['ms_per_step'])")"
timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4z/f.json 2>>gpurun_out/r4z/bench.log || exit 4
echo "mlp8192 100: $(python -c "import json;print(json.load(open('gpurun_out/r4z/f.json'))['ms_per_step'])")"
timeout -k 10 120 python bench.py --config mlp8192 --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4z/fd.json 2>>gpurun_out/r4z/bench.log || exit 4
echo "mlp8192 driver cmd: $(python -c "import json;print(json.load(open('gpurun_out/r4z/fd.json'))['ms_per_step'])")"
bash tools/prof_step.sh r4_final_mlp4 --steps 30 --warmup 10 || exit 5
python tools/prof_timeline.py gpurun_out/prof_r4_final_mlp4 > gpurun_out/r4z/tl_mlp4.txt 2>&1
bash tools/prof_step.sh r4_final_f8 --config mlp8192 --steps 30 --warmup 10 || exit 5
python tools/prof_timeline.py gpurun_out/prof_r4_final_f8 > gpurun_out/r4z/tl_f8.txt 2>&1
tail -14 gpurun_out/r4z/tl_f8.txt
