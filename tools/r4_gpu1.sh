#!/bin/bash
mkdir -p gpurun_out/r4a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4a/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r4a/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r4a/gpu_tests.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4a/bench_drv.json 2>gpurun_out/r4a/bench_drv.log && cat gpurun_out/r4a/bench_drv.json
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 20 > gpurun_out/r4a/bench_100.json 2>>gpurun_out/r4a/bench_drv.log && cat gpurun_out/r4a/bench_100.json
timeout -k 10 300 python bench.py --config mlp8192 --steps 50 --warmup 10 > gpurun_out/r4a/bench_fp8.json 2>>gpurun_out/r4a/bench_drv.log && cat gpurun_out/r4a/bench_fp8.json
