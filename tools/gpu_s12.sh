set -e
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab_bench.sh "base=" "w128=PZ_GEMM_W128=1" "p128f=PZ_GEMM_P128=2" "p128=PZ_GEMM_P128=1" > gpurun_out/s12_ab.txt 2>&1 || { cat gpurun_out/s12_ab.txt; exit 1; }
cat gpurun_out/s12_ab.txt
