set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s6_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/s6_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/s6_gpu_tests.txt
grep -E "world [0-9] " gpurun_out/s6_gpu_tests.txt || true
timeout -k 10 300 python bench.py > gpurun_out/s6_bench.json 2>gpurun_out/s6_bench.log
cat gpurun_out/s6_bench.json
