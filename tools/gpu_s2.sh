set -e
mkdir -p gpurun_out
ROUNDS=2 ARGS="--config deep16x8192 --steps 20 --warmup 5" bash tools/ab_bench.sh "fuse=PZ_OPT_FUSE=1" "sep=PZ_OPT_FUSE=0" > gpurun_out/s2_ab_deep.txt 2>&1 || { cat gpurun_out/s2_ab_deep.txt; exit 1; }
cat gpurun_out/s2_ab_deep.txt
ROUNDS=2 ARGS="--config mlp4x8192 --steps 40 --warmup 10" bash tools/ab_bench.sh "fuse=PZ_OPT_FUSE=1" "sep=PZ_OPT_FUSE=0" > gpurun_out/s2_ab_4x8192.txt 2>&1 || { cat gpurun_out/s2_ab_4x8192.txt; exit 1; }
cat gpurun_out/s2_ab_4x8192.txt
ROUNDS=2 ARGS="--config mlp8192_bf16" bash tools/ab_bench.sh "fuse=PZ_OPT_FUSE=1" "sep=PZ_OPT_FUSE=0" > gpurun_out/s2_ab_8192.txt 2>&1 || { cat gpurun_out/s2_ab_8192.txt; exit 1; }
cat gpurun_out/s2_ab_8192.txt
