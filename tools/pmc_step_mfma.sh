#!/bin/bash
# In-step MFMA utilisation per kernel: one rocprofv3 --pmc pass (kernel trace only) over a short
# bench.py run; summarise with `python tools/pmc_step_mfma_summary.py gpurun_out/pmc_step_mfma`.
set -e
repo=$(pwd)
out=$repo/gpurun_out/pmc_step_mfma
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$out" -o run --output-format csv \
    -- python3 "$repo/bench.py" --steps 10 --warmup 3 > "$out.log" 2>&1
