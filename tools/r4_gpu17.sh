#!/bin/bash
# r4: fp8 copy straight from fp32 when the bf16 output is not stored (D8): kernel + engine tests,
# stamps, fp8 step A/B (PZ_F8_D8=0/1)
mkdir -p gpurun_out/r4q
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_fastpaths_gpu.py -v --timeout 300 --timeout-method thread -k "fp8 or relu or bitmask or natural" > gpurun_out/r4q/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " gpurun_out/r4q/tests.txt | cut -c1-250 | tail -50
[ $rc -le 1 ] || exit 2
timeout -k 10 300 scratch/gemm_stamps f8n_fwd_L1_o8 f8n_fwd_L1_d8 f8n_fwd_L1_2wg_o8 f8n_fwd_L1_2wg_d8 f8_dX_L2_2wg_o8 f8_dX_L2_2wg_d8 > gpurun_out/r4q/stamps.txt 2>&1 || exit 3
cat gpurun_out/r4q/stamps.txt
for i in 1 2; do
  for d in 1 0; do
    PZ_F8_D8=$d timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4q/f.json 2>>gpurun_out/r4q/bench.log || exit 4
    echo "mlp8192 PZ_F8_D8=$d: $(python -c "import json;print(json.load(open('gpurun_out/r4q/f.json'))['ms_per_step'])")"
  done
done
