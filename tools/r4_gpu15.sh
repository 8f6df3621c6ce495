#!/bin/bash
# r4: GEMMs vs hipBLASLt (bf16 + fp8 cases), every bench config, split-K stamps
mkdir -p gpurun_out/r4o
timeout -k 10 600 python tools/gemm_bench.py fwd_L1 fwd_L2 fwd_L3 dX_L3 dX_L2 dW_L3 dW_L2 dW_L1 f8_8k_L1 f8_8k_L2 f8_fwd_L2 f8n_8k_L1 f8_8k_dX > gpurun_out/r4o/gemm_bench.txt 2>&1 || exit 2
grep -v "^{" gpurun_out/r4o/gemm_bench.txt | tail -14
timeout -k 10 300 scratch/gemm_stamps fwd_L3_fx dW_L3 dW_L1 dW_L2 fwd_L1_s0_fx fwd_L2_fx dX_L2 f8n_fwd_L1_fx f8_dW_L2 > gpurun_out/r4o/stamps.txt 2>&1 || exit 3
bash tools/bench_all.sh r4 > gpurun_out/r4o/bench_all.txt 2>&1 || exit 4
tail -12 gpurun_out/r4o/bench_all.txt
PZ_COV_GPU=1 PZ_LINECOV_MISSING=1 timeout -k 10 900 python -u tools/line_coverage.py tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r4o/cov.txt 2>&1
echo "cov rc=$?"; grep -E "passed|failed|TOTAL|functional" gpurun_out/r4o/cov.txt | cut -c1-300 | head -6
