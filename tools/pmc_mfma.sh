#!/bin/bash
# MFMA-pipe utilisation of the GEMM main loop: one rocprofv3 --pmc pass (kernel trace only,
# never combined with sys/runtime traces) per tools/gemm_lab case; summarise with
# `python tools/pmc_mfma_summary.py gpurun_out/pmc_mfma`.
# usage: tools/pmc_mfma.sh [case ...]   (default: fwd_L2 dX_L2 dW_L2 fwd_L1 dX_L3)
set -e
repo=$(pwd)
out=$repo/gpurun_out/pmc_mfma
mkdir -p "$out"
cases=${*:-fwd_L2 dX_L2 dW_L2 fwd_L1 dX_L3}
for c in $cases; do
  (cd /tmp && export TMPDIR=/tmp && LAB_ROUNDS=2 timeout -k 10 120 rocprofv3 --kernel-trace \
      --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_ANY SQ_WAVES \
      -d "$out/$c" -o run --output-format csv -- "$repo/tools/gemm_lab" "$c") > "$out/$c.log" 2>&1
done
