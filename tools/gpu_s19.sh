set -e
mkdir -p gpurun_out
ROUNDS=3 ARGS="--config mlp8192" bash tools/ab_bench.sh "g256=PZ_QUANT_GRID=256" "g512=PZ_QUANT_GRID=512" "g2048=PZ_QUANT_GRID=2048" > gpurun_out/s19_ab.txt 2>&1 || { cat gpurun_out/s19_ab.txt; exit 1; }
cat gpurun_out/s19_ab.txt
