#!/bin/bash
# round-6 session: steady state over a long run (mlp4, 500 steps after 20 warm-up, per-step GPU periods)
set -e
out=gpurun_out/r6d18
mkdir -p $out
PZ_BENCH_SERIES=1 timeout -k 10 300 python bench.py --steps 500 --warmup 20 > $out/bench500.txt 2>&1 || { tail -20 $out/bench500.txt; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $out/bench500.txt
python3 - $out/bench500.txt <<'PY'
import sys, statistics
for l in open(sys.argv[1]):
    if "step periods" in l:
        v = [float(x) for x in l.split("(ms):")[1].split()][20:]
        v.sort()
        print(f"timed steps {len(v)}: median {statistics.median(v):.4f} p10 {v[len(v)//10]:.4f} p90 {v[9*len(v)//10]:.4f} max {v[-1]:.4f} ms")
PY
