#!/bin/bash
# round-6 session: data-parallel equivalence tests with the "mid" sharded-optimizer scope
set -e
out=gpurun_out/r6d5
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_dp_gpu.py -x -v --timeout 240 --timeout-method thread > $out/dp_tests.txt 2>&1 || { tail -40 $out/dp_tests.txt; exit 1; }
tail -3 $out/dp_tests.txt
