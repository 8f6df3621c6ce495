#!/bin/bash
mkdir -p gpurun_out/r4i
timeout -k 10 700 python -u -m pytest tests/test_fastpaths_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -v --timeout 300 --timeout-method thread -k "fastpaths or paired or write_through or torch_backward" > gpurun_out/r4i/tests.txt 2>&1
grep -E "PASS|FAIL|^E  " gpurun_out/r4i/tests.txt | cut -c1-220 | tail -24
timeout -k 10 600 python tools/diag_dw_error.py > gpurun_out/r4i/diag.txt 2>&1; cat gpurun_out/r4i/diag.txt | cut -c1-400
bash tools/r4_gpu8.sh
