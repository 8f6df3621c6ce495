set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s20_tests.txt 2>&1 || { tail -30 gpurun_out/s20_tests.txt; exit 1; }
tail -1 gpurun_out/s20_tests.txt
ROUNDS=3 ARGS="--config mlp8192" bash tools/ab_bench.sh "qt16=" > gpurun_out/s20_ab.txt 2>&1 || { cat gpurun_out/s20_ab.txt; exit 1; }
cat gpurun_out/s20_ab.txt
bash tools/prof_step.sh f8t --config mlp8192 --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_f8t > gpurun_out/prof_f8t_timeline.txt
grep -E "quantize|quant_transpose|step:" gpurun_out/prof_f8t_timeline.txt
