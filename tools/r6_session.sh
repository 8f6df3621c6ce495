#!/bin/bash
# round-6 session: per-kernel HBM traffic of the mlp4 step (two rocprofv3 --pmc passes, kernel trace only)
set -e
repo=$(pwd)
out=$repo/gpurun_out/pmc_step
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$out/f" -o run --output-format csv \
  -- python3 "$repo/bench.py" --steps 6 --warmup 3 > "$out/f.log" 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$out/w" -o run --output-format csv \
  -- python3 "$repo/bench.py" --steps 6 --warmup 3 > "$out/w.log" 2>&1
cd "$repo"
python3 tools/pmc_step_summary.py gpurun_out/pmc_step > gpurun_out/pmc_step/summary.txt 2>&1 || true
head -30 gpurun_out/pmc_step/summary.txt
