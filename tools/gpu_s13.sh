set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s13_tests.txt 2>&1 || { tail -30 gpurun_out/s13_tests.txt; exit 1; }
PZ_OPT_DEFER=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "dense or graph or fp8" >> gpurun_out/s13_tests.txt 2>&1 || { tail -30 gpurun_out/s13_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/s13_tests.txt
ROUNDS=3 bash tools/ab_bench.sh "base=" "defer=PZ_OPT_DEFER=1" > gpurun_out/s13_ab.txt 2>&1 || { cat gpurun_out/s13_ab.txt; exit 1; }
cat gpurun_out/s13_ab.txt
ROUNDS=2 ARGS="--config mlp8192" bash tools/ab_bench.sh "base=" "defer=PZ_OPT_DEFER=1" > gpurun_out/s13_ab_f8.txt 2>&1 || { cat gpurun_out/s13_ab_f8.txt; exit 1; }
cat gpurun_out/s13_ab_f8.txt
PZ_OPT_DEFER=1 bash tools/prof_step.sh defer --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_defer > gpurun_out/prof_defer_timeline.txt
cat gpurun_out/prof_defer_timeline.txt
