#!/bin/bash
# round-6 GPU call 1: driver bench, 100-step bench, hipBLASLt kernel names for the step shapes
set -e
repo=$(pwd)
mkdir -p gpurun_out/r6c1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6c1/bench_driver.json 2>gpurun_out/r6c1/bench_driver.log
cat gpurun_out/r6c1/bench_driver.json
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/r6c1/bench100.json 2>gpurun_out/r6c1/bench100.log
cat gpurun_out/r6c1/bench100.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$repo/gpurun_out/r6c1/hbl" -o hbl -- python3 "$repo/tools/hipblaslt_kernels.py" > "$repo/gpurun_out/r6c1/hbl.log" 2>&1
find "$repo/gpurun_out/r6c1/hbl" -name "*.csv"
