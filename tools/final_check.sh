#!/bin/bash
# Round-end check on one MI355X: GPU test tier, smoke(), the headline bench, a kernel-trace profile.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu_tests.txt 2>&1
tail -1 gpurun_out/final_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1
tail -1 gpurun_out/final_smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench_driver.json 2>gpurun_out/final_bench_driver.log
cat gpurun_out/final_bench_driver.json
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2>gpurun_out/final_bench.log
cat gpurun_out/final_bench.json
timeout -k 10 300 python bench.py --config mlp8192 --steps 50 --warmup 10 > gpurun_out/final_bench_fp8.json 2>gpurun_out/final_bench_fp8.log
cat gpurun_out/final_bench_fp8.json
tools/prof_step.sh final --steps 30 --warmup 10
python tools/prof_summary.py gpurun_out/prof_final > gpurun_out/prof_final_summary.txt 2>&1
tail -14 gpurun_out/prof_final_summary.txt
