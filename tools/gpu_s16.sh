set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s16_tests.txt 2>&1 || { tail -30 gpurun_out/s16_tests.txt; exit 1; }
tail -1 gpurun_out/s16_tests.txt
timeout -k 10 300 python tools/gemm_bench.py fwdL1_bias fwdL1_mask fwd_L2 fwd_L3 f8_8k_L1 f8_8k_L2 bf_8k_L1 2>&1 | grep -v amdgpu.ids | grep -v "^{"
ROUNDS=3 bash tools/ab_bench.sh "bias_early=" > gpurun_out/s16_ab.txt 2>&1 || { cat gpurun_out/s16_ab.txt; exit 1; }
cat gpurun_out/s16_ab.txt
ROUNDS=2 ARGS="--config mlp8192" bash tools/ab_bench.sh "bias_early_f8=" >> gpurun_out/s16_ab.txt 2>&1 || { cat gpurun_out/s16_ab.txt; exit 1; }
tail -2 gpurun_out/s16_ab.txt
