#!/bin/bash
# r4 lab: VAR 30 with / without the s_setprio bracket around the ping-pong MFMA block, interleaved x2
mkdir -p gpurun_out/r4s
for i in 1 2; do
  timeout -k 10 300 scratch/gemm_stamps dX_L2 dX_L2_np fwd_L2 fwd_L2_np dW_L2 dW_L2_np > gpurun_out/r4s/stamps$i.txt 2>&1 || exit 3
  grep -v "epilogue (wave" gpurun_out/r4s/stamps$i.txt | cut -c1-150
done
