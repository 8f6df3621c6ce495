#!/bin/bash
mkdir -p gpurun_out/r4y
timeout -k 10 1000 python -u tools/grad_dtype_convergence.py --fp8 --steps 600 > gpurun_out/r4y/conv_fp8.txt 2>&1 || exit 2
cat gpurun_out/r4y/conv_fp8.txt
