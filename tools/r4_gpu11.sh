#!/bin/bash
# r4: fp8 activation-scale parity fix tests, step profiles (mlp4, DP schedule at world 1, fp8), epilogue
# stamps by epilogue kind, driver-command bench
mkdir -p gpurun_out/r4k
timeout -k 10 900 python -u -m pytest tests/test_fastpaths_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -v --timeout 300 --timeout-method thread -k "fastpaths or fp8 or xent or head or graph" > gpurun_out/r4k/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " gpurun_out/r4k/tests.txt | cut -c1-300 | tail -40
[ $rc -le 1 ] || exit 2
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4k/drv.json 2>>gpurun_out/r4k/bench.log || exit 3
  echo "driver cmd mlp4: $(python -c "import json;print(json.load(open('gpurun_out/r4k/drv.json'))['ms_per_step'])")"
  timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4k/m.json 2>>gpurun_out/r4k/bench.log || exit 3
  echo "mlp4 100: $(python -c "import json;print(json.load(open('gpurun_out/r4k/m.json'))['ms_per_step'])")"
  timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4k/f.json 2>>gpurun_out/r4k/bench.log || exit 3
  echo "mlp8192 100: $(python -c "import json;print(json.load(open('gpurun_out/r4k/f.json'))['ms_per_step'])")"
done
bash tools/prof_step.sh r4_mlp4 --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_mlp4 > gpurun_out/r4k/tl_mlp4.txt 2>&1
PZ_FORCE_COMM=1 PZ_COMM=proxy PZ_COMM_PROXY_GBPS=1e12 bash tools/prof_step.sh r4_dpnone --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_dpnone > gpurun_out/r4k/tl_dpnone.txt 2>&1
bash tools/prof_step.sh r4_f8 --config mlp8192 --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_f8 > gpurun_out/r4k/tl_f8.txt 2>&1
timeout -k 10 300 scratch/gemm_stamps fwd_L1 fwdL1_m9 fwdL1_m8 fwdL1_m7 fwdL1_m4 fwdL1_m5 fwdL1_st dX_L3 > gpurun_out/r4k/stamps.txt 2>&1 || exit 5
tail -20 gpurun_out/r4k/tl_dpnone.txt
