#!/bin/bash
# full GPU test tier (one pytest process) + smoke, as the driver runs them at round end
set -e
out=gpurun_out/r6tier
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.txt 2>&1 || { tail -40 $out/tests.txt; exit 1; }
tail -3 $out/tests.txt
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
