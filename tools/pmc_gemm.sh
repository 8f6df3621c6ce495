#!/bin/bash
# Hardware-counter passes over tools/gemm_bench.py cases (one rocprofv3 run per counter group,
# kernel-trace only: never combined with sys/runtime traces). Summarise with
# `python tools/pmc_summary.py gpurun_out/pmc_<tag>`.
# usage: PMC_SET=core|mem [PMC_PROG=tools/sk_bench.py] tools/pmc_gemm.sh <tag> <bench args>...
set -e
tag=$1; shift
out=$(pwd)/gpurun_out/pmc_$tag
mkdir -p "$out"
if [ "${PMC_SET:-core}" = "core" ]; then
  groups=(
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
    "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
  )
else
  groups=(
    "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ GRBM_GUI_ACTIVE"
    "TA_BUSY_avr TD_TC_STALL TCP_TCP_TA_DATA_STALL_CYCLES TCP_LFIFO_STALL_CYCLES GRBM_GUI_ACTIVE"
    "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
  )
fi
repo=$(pwd)
i=0
for g in "${groups[@]}"; do
  i=$((i + 1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --pmc $g -d "$out/g$i" -o run \
      -- python3 "$repo/${PMC_PROG:-tools/gemm_bench.py}" "$@") > "$out/g$i.log" 2>&1
done
