# usage: tools/bench_all.sh [tag]   (every bench.py config on one GPU + the PyTorch eager baseline)
set -e
tag=${1:-r3}
mkdir -p gpurun_out
out=gpurun_out/bench_all_$tag.jsonl
: > $out
for c in mlp4 mlp8192 mlp8192_bf16 mlp4x8192 mlp4_fp32 mlp4_fp64; do
  timeout -k 10 240 python bench.py --config $c --steps 50 --warmup 10 2>/dev/null | tail -1 >> $out
  echo "$c done"
done
timeout -k 10 300 python bench.py --config deep16x8192 --steps 20 --warmup 5 2>/dev/null | tail -1 >> $out
timeout -k 10 240 python tools/torch_eager_baseline.py > gpurun_out/eager_$tag.json 2>/dev/null
cat $out | python -c "import json,sys; [print(d['config']['model'], d['dtype'], d['ms_per_step'], d['value']) for d in map(json.loads, sys.stdin)]"
tail -2 gpurun_out/eager_$tag.json
