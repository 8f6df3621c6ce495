#!/bin/bash
# r4: device-scope events (PZ_TORCH_EVENTS A/B), DP schedule after the chunk change, engine tests
mkdir -p gpurun_out/r4l
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_fastpaths_gpu.py tests/test_dp_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r4l/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E  " gpurun_out/r4l/tests.txt | cut -c1-200 | tail -60
[ $rc -le 1 ] || exit 2
for i in 1 2; do
  for env in "PZ_TORCH_EVENTS=0" "PZ_TORCH_EVENTS=1"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4l/m.json 2>>gpurun_out/r4l/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4l/m.json'))['ms_per_step'])")"
    env $env timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4l/d.json 2>>gpurun_out/r4l/bench.log || exit 3
    echo "mlp4 driver $env: $(python -c "import json;print(json.load(open('gpurun_out/r4l/d.json'))['ms_per_step'])")"
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4l/f.json 2>>gpurun_out/r4l/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4l/f.json'))['ms_per_step'])")"
    env $env PZ_FORCE_COMM=1 PZ_COMM=proxy PZ_COMM_PROXY_GBPS=1e12 timeout -k 10 120 python bench.py --steps 60 --warmup 20 > gpurun_out/r4l/p.json 2>>gpurun_out/r4l/bench.log || exit 3
    echo "mlp4 dpnone $env: $(python -c "import json;print(json.load(open('gpurun_out/r4l/p.json'))['ms_per_step'])")"
    env $env PZ_FORCE_COMM=1 PZ_COMM=torch timeout -k 10 120 python bench.py --steps 60 --warmup 20 > gpurun_out/r4l/t.json 2>>gpurun_out/r4l/bench.log || exit 3
    echo "mlp4 torch-comm $env: $(python -c "import json;print(json.load(open('gpurun_out/r4l/t.json'))['ms_per_step'])")"
  done
done
bash tools/prof_step.sh r4_ev_mlp4 --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_ev_mlp4 > gpurun_out/r4l/tl_mlp4.txt 2>&1
PZ_FORCE_COMM=1 PZ_COMM=proxy PZ_COMM_PROXY_GBPS=1e12 bash tools/prof_step.sh r4_ev_dpnone --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_ev_dpnone > gpurun_out/r4l/tl_dpnone.txt 2>&1
tail -22 gpurun_out/r4l/tl_mlp4.txt
