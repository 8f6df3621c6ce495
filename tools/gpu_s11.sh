set -e
mkdir -p gpurun_out
ROUNDS=3 ARGS="--steps 60 --warmup 15" bash tools/ab_bench.sh "native=PZ_FORCE_COMM=1,PZ_COMM=native" "torch=PZ_FORCE_COMM=1,PZ_COMM=torch" "nocomm=" > gpurun_out/s11_ab.txt 2>&1 || { cat gpurun_out/s11_ab.txt; exit 1; }
cat gpurun_out/s11_ab.txt
