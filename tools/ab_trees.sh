#!/bin/bash
# Same-box A/B of two source trees (e.g. a git worktree of an earlier commit in ./ab_base):
# bench.py runs alternate between the trees, interleaved rounds.
# usage: ROUNDS=3 ARGS="--steps 20 --warmup 5" tools/ab_trees.sh ab_base .
rounds=${ROUNDS:-3}
args=${ARGS:---steps 100 --warmup 20}
for r in $(seq 1 "$rounds"); do
  for tree in "$@"; do
    out=$(cd "$tree" && timeout -k 10 300 python bench.py $args 2>/dev/null) || { echo "$tree FAILED"; exit 1; }
    ms=$(echo "$out" | python -c "import json,sys; print(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'])")
    echo "round $r $tree ms_per_step $ms"
  done
done
