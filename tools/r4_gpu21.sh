#!/bin/bash
# r4: ping-pong MFMA blocks with / without s_setprio (PZ_GEMM_PRIO), step A/B interleaved x3
mkdir -p gpurun_out/r4t
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "relu or split_k or pair" > gpurun_out/r4t/tests.txt 2>&1
rc=$?; tail -1 gpurun_out/r4t/tests.txt; [ $rc -le 1 ] || exit 2
for i in 1 2 3; do
  for pr in 1 0; do
    PZ_GEMM_PRIO=$pr timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4t/m.json 2>>gpurun_out/r4t/bench.log || exit 3
    echo "mlp4 PZ_GEMM_PRIO=$pr: $(python -c "import json;print(json.load(open('gpurun_out/r4t/m.json'))['ms_per_step'])")"
    PZ_GEMM_PRIO=$pr timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4t/f.json 2>>gpurun_out/r4t/bench.log || exit 3
    echo "mlp8192 PZ_GEMM_PRIO=$pr: $(python -c "import json;print(json.load(open('gpurun_out/r4t/f.json'))['ms_per_step'])")"
  done
done
