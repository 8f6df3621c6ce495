#!/bin/bash
# round-6 final check on one MI355X: GPU tier, smoke, the driver's bench command, a 100-step run, every
# bench config (50 steps), 2-rank gloo rehearsal of the DP bench path
set -e
out=gpurun_out/r6final
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/tests.txt 2>&1 || { tail -40 $out/tests.txt; exit 1; }
tail -1 $out/tests.txt
timeout -k 10 300 python __graft_entry__.py smoke > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench_driver.txt 2>&1 || { tail -20 $out/bench_driver.txt; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/bench_driver.txt | sed 's/^/driver /'
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > $out/bench100.txt 2>&1 || { tail -20 $out/bench100.txt; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/bench100.txt | sed 's/^/100-step /'
: > $out/all_configs.jsonl
for c in mlp8192 mlp8192_bf16 mlp4x8192 mlp4_fp32 deep16x8192; do
  timeout -k 10 400 python bench.py --config $c --steps 50 --warmup 10 > $out/bench_$c.txt 2>&1 || { tail -20 $out/bench_$c.txt; exit 1; }
  grep '"metric"' $out/bench_$c.txt >> $out/all_configs.jsonl
  grep -o '"ms_per_step": [0-9.]*' $out/bench_$c.txt | sed "s/^/$c /"
done
