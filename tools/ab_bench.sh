#!/bin/bash
# Same-box A/B of bench.py under environment variants, interleaved rounds (guide §5.4 rule 24).
# usage: ROUNDS=3 ARGS="--steps 100 --warmup 20" tools/ab_bench.sh "NAME=ENV1=a,ENV2=b" "base=" ...
mkdir -p gpurun_out
rounds=${ROUNDS:-3}
args=${ARGS:---steps 100 --warmup 20}
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name="${spec%%=*}"; envs="${spec#*=}"
    envcmd=()
    IFS=',' read -ra kv <<< "$envs"
    for e in "${kv[@]}"; do [ -n "$e" ] && envcmd+=("$e"); done
    out=$(env "${envcmd[@]}" timeout -k 10 300 python bench.py $args 2>/dev/null) || { echo "$name FAILED rc=$?"; exit 1; }
    ms=$(echo "$out" | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])")
    echo "round $r $name ms_per_step $ms"
  done
done
