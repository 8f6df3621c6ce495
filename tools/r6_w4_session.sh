set -o pipefail
mkdir -p gpurun_out/w4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "w4_dx or mfma_layouts or relu_bitmask or identity" > gpurun_out/w4/tests.txt 2>&1 || { tail -30 gpurun_out/w4/tests.txt; exit 1; }
tail -3 gpurun_out/w4/tests.txt
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/w4/gb_on.txt 2>&1 && PZ_GEMM_W4=0 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/w4/gb_off.txt 2>&1 && grep -h "dX\|fwd_L2" gpurun_out/w4/gb_on.txt gpurun_out/w4/gb_off.txt | grep -v "^{"
for i in 1 2; do timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/w4/bench_on$i.txt 2>&1 && PZ_GEMM_W4=0 timeout -k 10 200 python bench.py --steps 50 --warmup 10 > gpurun_out/w4/bench_off$i.txt 2>&1 || exit 1; done
grep -ho '"ms_per_step": [0-9.]*' gpurun_out/w4/bench_on*.txt gpurun_out/w4/bench_off*.txt
