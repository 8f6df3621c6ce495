#!/bin/bash
mkdir -p gpurun_out/r4b
timeout -k 10 900 python -u -m pytest tests/test_fastpaths_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4b/fastpaths.txt 2>&1
rc=$?; tail -25 gpurun_out/r4b/fastpaths.txt; exit $rc
