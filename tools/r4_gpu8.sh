#!/bin/bash
# r4: counters (dX vs hipBLASLt, in-step MFMA busy), comm pressure, fp32-gradient headline, W128 skinny fwd
mkdir -p gpurun_out/r4h
bash tools/r4_pmc.sh > gpurun_out/r4h/pmc.log 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/r4h/pmc.log
for i in 1 2; do
  for env in "PZ_GRAD_DTYPE=bf16" "PZ_GRAD_DTYPE=fp32" "PZ_GEMM_W128=1"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4h/m.json 2>>gpurun_out/r4h/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4h/m.json'))['ms_per_step'])")"
  done
done
timeout -k 10 900 python tools/comm_pressure.py --rounds 2 --steps 50 > gpurun_out/r4h/comm_pressure.txt 2>&1; echo "comm rc=$?"
tail -9 gpurun_out/r4h/comm_pressure.txt
