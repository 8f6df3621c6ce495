set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/s8_tests.txt 2>&1 || { tail -60 gpurun_out/s8_tests.txt; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/s8_tests.txt | tail -15
ROUNDS=2 bash tools/ab_bench.sh "forced_native=PZ_FORCE_COMM=1,PZ_COMM=native" "forced_torch=PZ_FORCE_COMM=1,PZ_COMM=torch" "nocomm=" > gpurun_out/s8_ab.txt 2>&1 || { cat gpurun_out/s8_ab.txt; exit 1; }
cat gpurun_out/s8_ab.txt
