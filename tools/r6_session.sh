#!/bin/bash
# round-6 GPU call: DP / sharded-optimizer tests, stream-K + pair tests
set -e
mkdir -p gpurun_out/r6c2
timeout -k 10 900 python -u -m pytest tests/test_dp_gpu.py tests/test_gemm_sk_gpu.py -x -v --timeout 300 --timeout-method thread -k "not bench_launches" > gpurun_out/r6c2/dp_tests.txt 2>&1 || { tail -60 gpurun_out/r6c2/dp_tests.txt; exit 1; }
tail -40 gpurun_out/r6c2/dp_tests.txt
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "pair" > gpurun_out/r6c2/pair_tests.txt 2>&1 || { tail -40 gpurun_out/r6c2/pair_tests.txt; exit 1; }
tail -3 gpurun_out/r6c2/pair_tests.txt
