#!/bin/bash
# r4: store-policy / optimizer-stream A/B, fp32-gradient headline, W128 skinny fwd; then counters
mkdir -p gpurun_out/r4h
for i in 1 2; do
  for env in "PZ_GEMM_WT=0" "PZ_GEMM_WT=1" "PZ_OPT_NT=1" "PZ_GEMM_WT=1 PZ_OPT_NT=1" "PZ_GRAD_DTYPE=fp32" "PZ_GEMM_W128=1"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4h/m.json 2>>gpurun_out/r4h/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4h/m.json'))['ms_per_step'])")"
  done
  for env in "PZ_GEMM_WT=0" "PZ_GEMM_WT=1" "PZ_OPT_NT=1"; do
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4h/f.json 2>>gpurun_out/r4h/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4h/f.json'))['ms_per_step'])")"
  done
done
bash tools/r4_pmc.sh > gpurun_out/r4h/pmc.log 2>&1; echo "pmc rc=$?"; tail -5 gpurun_out/r4h/pmc.log
