#!/bin/bash
# r4 counters: pz dX_L2 vs hipBLASLt dX_L2 (two --pmc passes, kernel trace only), in-step MFMA busy
set -e
mkdir -p gpurun_out/r4p
PMC_SET=core bash tools/pmc_gemm.sh dxl2 dX_L2 dX_L3 fwd_L2
python tools/pmc_summary.py gpurun_out/pmc_dxl2 > gpurun_out/r4p/pmc_dx_vs_hipblaslt.txt 2>&1
bash tools/pmc_step_mfma.sh
python tools/pmc_step_mfma_summary.py gpurun_out/pmc_step_mfma > gpurun_out/r4p/pmc_step_mfma.txt 2>&1
head -60 gpurun_out/r4p/pmc_dx_vs_hipblaslt.txt
head -20 gpurun_out/r4p/pmc_step_mfma.txt
