set -e
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab_bench.sh "base=" "g16=PZ_GRAD_DTYPE=bf16" "prio0=PZ_OPT_PRIO=0" > gpurun_out/s5_ab.txt 2>&1 || { cat gpurun_out/s5_ab.txt; exit 1; }
cat gpurun_out/s5_ab.txt
ROUNDS=2 ARGS="--config mlp8192" bash tools/ab_bench.sh "base=" "g16=PZ_GRAD_DTYPE=bf16" "prio0=PZ_OPT_PRIO=0" > gpurun_out/s5_ab_f8.txt 2>&1 || { cat gpurun_out/s5_ab_f8.txt; exit 1; }
cat gpurun_out/s5_ab_f8.txt
