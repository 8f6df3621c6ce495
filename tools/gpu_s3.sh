set -e
mkdir -p gpurun_out
bash tools/prof_step.sh f8 --config mlp8192 --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_f8 > gpurun_out/prof_f8_timeline.txt
cat gpurun_out/prof_f8_timeline.txt
bash tools/prof_step.sh bf8192 --config mlp8192_bf16 --steps 30 --warmup 10
python tools/prof_timeline.py gpurun_out/prof_bf8192 > gpurun_out/prof_bf8192_timeline.txt
cat gpurun_out/prof_bf8192_timeline.txt
