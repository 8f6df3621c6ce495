set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s15_tests.txt 2>&1 || { tail -30 gpurun_out/s15_tests.txt; exit 1; }
tail -1 gpurun_out/s15_tests.txt
timeout -k 10 300 python tools/gemm_bench.py fwd_L1 fwdL1_mask fwdL1_mask0 fwdL2_mask f8_8k_L1 bf_8k_L1 2>&1 | grep -v amdgpu.ids | grep -v "^{"
ROUNDS=3 bash tools/ab_bench.sh "comb=" > gpurun_out/s15_ab.txt 2>&1 || { cat gpurun_out/s15_ab.txt; exit 1; }
cat gpurun_out/s15_ab.txt
ROUNDS=2 ARGS="--config mlp8192" bash tools/ab_bench.sh "comb_f8=" >> gpurun_out/s15_ab.txt 2>&1 || { cat gpurun_out/s15_ab.txt; exit 1; }
tail -2 gpurun_out/s15_ab.txt
