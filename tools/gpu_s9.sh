set -e
mkdir -p gpurun_out
PZ_FORCE_COMM=1 PZ_COMM=native bash tools/prof_step.sh cnat --steps 20 --warmup 5
python tools/prof_timeline.py gpurun_out/prof_cnat > gpurun_out/prof_cnat_timeline.txt
cat gpurun_out/prof_cnat_timeline.txt
PZ_FORCE_COMM=1 PZ_COMM=torch bash tools/prof_step.sh ctorch --steps 20 --warmup 5
python tools/prof_timeline.py gpurun_out/prof_ctorch > gpurun_out/prof_ctorch_timeline.txt
cat gpurun_out/prof_ctorch_timeline.txt
