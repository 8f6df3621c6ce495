set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s7_tests.txt 2>&1 || { tail -40 gpurun_out/s7_tests.txt; exit 1; }
tail -2 gpurun_out/s7_tests.txt
ROUNDS=3 bash tools/ab_bench.sh "pf=PZ_PREFETCH=1" "nopf=PZ_PREFETCH=0" > gpurun_out/s7_ab.txt 2>&1 || { cat gpurun_out/s7_ab.txt; exit 1; }
cat gpurun_out/s7_ab.txt
bash tools/prof_step.sh pf --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_pf > gpurun_out/prof_pf_timeline.txt
cat gpurun_out/prof_pf_timeline.txt
