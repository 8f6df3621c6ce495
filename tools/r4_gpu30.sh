#!/bin/bash
# r4: device-side signals with a slow poll (s_sleep 64): is the GEMM slowdown beside a resident waiter the poll rate?
mkdir -p gpurun_out/r4t
for env in "PZ_DEV_SIG=0" "PZ_DEV_SIG=1"; do
  env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4t/m.json 2>>gpurun_out/r4t/bench.log || exit 3
  echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4t/m.json'))['ms_per_step'])")"
done
PZ_DEV_SIG=1 bash tools/prof_step.sh r4_sig2_mlp4 --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_sig2_mlp4 > gpurun_out/r4t/tl_mlp4.txt 2>&1
rm -rf gpurun_out/prof_r4_sig2_mlp4
tail -26 gpurun_out/r4t/tl_mlp4.txt
