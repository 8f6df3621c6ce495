#!/bin/bash
# r4: re-tolerated gradient tests, NT/WT default-on + PZ_PAIR_SIDE A/B, DP comm pressure, stamps
mkdir -p gpurun_out/r4j
timeout -k 10 900 python -u -m pytest tests/test_fastpaths_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -v --timeout 300 --timeout-method thread -k "sgd_curve or matches_fp32_torch or write_through or pair or bitmask or relu or fp8 or epilogue" > gpurun_out/r4j/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " gpurun_out/r4j/tests.txt | cut -c1-400 | tail -24
[ $rc -le 1 ] || exit 2  # test failures go on; a crash / timeout ends the call
for i in 1 2; do
  for env in "PZ_PAIR_SIDE=1" "PZ_PAIR_SIDE=0" "PZ_GEMM_WT=0 PZ_OPT_NT=0"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4j/m.json 2>>gpurun_out/r4j/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4j/m.json'))['ms_per_step'])")"
  done
  for env in "PZ_PAIR_SIDE=1" "PZ_PAIR_SIDE=0"; do
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4j/f.json 2>>gpurun_out/r4j/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4j/f.json'))['ms_per_step'])")"
  done
done
timeout -k 10 300 scratch/gemm_stamps fwd_L1 fwd_L2 fwd_L2_wt fwd_L2_fx dX_L2 dX_L2_wt f8n_fwd_L1_fx f8n_fwd_L1_fx_wt f8n_fwd_L1_2wg f8_dX_L2 f8_dX_L2_2wg > gpurun_out/r4j/stamps.txt 2>&1 || exit 4
timeout -k 10 900 python -u tools/comm_pressure.py --rounds 2 --steps 60 --ks 0,8,16,32 > gpurun_out/r4j/comm_pressure.txt 2>&1 || exit 5
tail -12 gpurun_out/r4j/comm_pressure.txt
