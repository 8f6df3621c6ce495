#!/bin/bash
# r4: LDS-array occupancy of the ping-pong main loop vs hipBLASLt (is the 8-wave 128x64 slice LDS-bound?),
# and the final tree's in-step MFMA busy
set -e
repo=$(pwd)
out=$repo/gpurun_out/pmc_lds
mkdir -p "$out"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d "$out/g1" -o run -- python3 "$repo/tools/gemm_bench.py" fwd_L2 dX_L2 dW_L2) > "$out/g1.log" 2>&1
echo "lds pass rc=$?"
python tools/pmc_db_summary.py gpurun_out/pmc_lds > gpurun_out/pmc_lds/summary.txt 2>&1 || true
head -40 gpurun_out/pmc_lds/summary.txt
bash tools/pmc_step_mfma.sh
python tools/pmc_step_mfma_summary.py gpurun_out/pmc_step_mfma > gpurun_out/pmc_step_mfma/summary_final.txt 2>&1
head -12 gpurun_out/pmc_step_mfma/summary_final.txt
