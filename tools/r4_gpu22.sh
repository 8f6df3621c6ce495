#!/bin/bash
mkdir -p gpurun_out/r4u
timeout -k 10 1000 python -u tools/grad_dtype_convergence.py --steps 400 > gpurun_out/r4u/conv.txt 2>&1 || exit 2
cat gpurun_out/r4u/conv.txt
