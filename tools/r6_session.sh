#!/bin/bash
# round-6 session: VAR 43 plain fp8 forward + the fp8 / w4 tests, fp8 mlp8192 and mlp4 bench with the final dispatch
set -e
out=gpurun_out/r6d11
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fastpaths_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp8 or w4 or layouts" > $out/tests.txt 2>&1 || { tail -30 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
for c in mlp8192 mlp4; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 20 > $out/bench_$c.txt 2>&1 || { tail -20 $out/bench_$c.txt; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.txt | sed "s/^/$c /"
done
timeout -k 10 300 python tools/gemm_bench.py > $out/gemm_bench.txt 2>&1 || true
grep -v "^{" $out/gemm_bench.txt | grep "TF" || true
