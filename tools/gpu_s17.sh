set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s17_tests.txt 2>&1 || { tail -30 gpurun_out/s17_tests.txt; exit 1; }
tail -1 gpurun_out/s17_tests.txt
timeout -k 10 300 python tools/gemm_bench.py fwdL1_nobias fwd_L3 f8_8k_L2 bf_8k_L2 2>&1 | grep -v amdgpu.ids | grep -v "^{"
ROUNDS=3 bash tools/ab_bench.sh "demote=" "fwd=PZ_EPI_DEMOTE=0" > gpurun_out/s17_ab.txt 2>&1 || { cat gpurun_out/s17_ab.txt; exit 1; }
cat gpurun_out/s17_ab.txt
ROUNDS=2 ARGS="--config mlp8192" bash tools/ab_bench.sh "demote_f8=" "fwd_f8=PZ_EPI_DEMOTE=0" >> gpurun_out/s17_ab.txt 2>&1 || { cat gpurun_out/s17_ab.txt; exit 1; }
tail -4 gpurun_out/s17_ab.txt
