set -e
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab_bench.sh "base=" "serial=PZ_OPT_OVERLAP=0" "nomerge=PZ_OPT_MERGE=0" "prio=PZ_OPT_PRIO=-1" > gpurun_out/s4_ab.txt 2>&1 || { cat gpurun_out/s4_ab.txt; exit 1; }
cat gpurun_out/s4_ab.txt
PZ_OPT_OVERLAP=0 bash tools/prof_step.sh serial --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_serial > gpurun_out/prof_serial_timeline.txt
cat gpurun_out/prof_serial_timeline.txt
