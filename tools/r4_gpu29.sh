#!/bin/bash
# r4: device-side stream signals (PZ_DEV_SIG A/B) — tests, same-box interleaved benches, step timeline
mkdir -p gpurun_out/r4s
timeout -k 10 400 python -u -m pytest tests/test_stream_signal_gpu.py -v -s --timeout 120 --timeout-method thread > gpurun_out/r4s/tests.txt 2>&1
rc=$?
grep -E "PASS|FAIL|^E  |vs event" gpurun_out/r4s/tests.txt | cut -c1-200 | tail -30
[ $rc -eq 0 ] || exit 2
for i in 1 2; do
  for env in "PZ_DEV_SIG=0" "PZ_DEV_SIG=1"; do
    env $env timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/r4s/m.json 2>>gpurun_out/r4s/bench.log || exit 3
    echo "mlp4 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4s/m.json'))['ms_per_step'])")"
    env $env timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4s/d.json 2>>gpurun_out/r4s/bench.log || exit 3
    echo "mlp4 driver $env: $(python -c "import json;print(json.load(open('gpurun_out/r4s/d.json'))['ms_per_step'])")"
    env $env timeout -k 10 120 python bench.py --config mlp8192 --steps 100 --warmup 20 > gpurun_out/r4s/f.json 2>>gpurun_out/r4s/bench.log || exit 3
    echo "mlp8192 $env: $(python -c "import json;print(json.load(open('gpurun_out/r4s/f.json'))['ms_per_step'])")"
  done
done
PZ_DEV_SIG=1 bash tools/prof_step.sh r4_sig_mlp4 --steps 30 --warmup 10 || exit 4
python tools/prof_timeline.py gpurun_out/prof_r4_sig_mlp4 > gpurun_out/r4s/tl_mlp4.txt 2>&1
rm -rf gpurun_out/prof_r4_sig_mlp4
tail -24 gpurun_out/r4s/tl_mlp4.txt
timeout -k 10 120 ./tools/packet_gap 200 1000 > gpurun_out/r4s/pg.txt 2>&1 && cat gpurun_out/r4s/pg.txt
