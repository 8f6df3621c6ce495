set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_update or engine or fused or graph or dense or fp8 or record" > gpurun_out/s1_tests.txt 2>&1 || { tail -40 gpurun_out/s1_tests.txt; exit 1; }
tail -2 gpurun_out/s1_tests.txt
ROUNDS=3 bash tools/ab_bench.sh "fuse=PZ_OPT_FUSE=1" "sep=PZ_OPT_FUSE=0" > gpurun_out/s1_ab.txt 2>&1 || { cat gpurun_out/s1_ab.txt; exit 1; }
cat gpurun_out/s1_ab.txt
bash tools/prof_step.sh fuse --steps 30 --warmup 10
python tools/prof_summary.py gpurun_out/prof_fuse > gpurun_out/prof_fuse_summary.txt 2>&1
tail -14 gpurun_out/prof_fuse_summary.txt
