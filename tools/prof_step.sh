#!/bin/bash
# Kernel trace + stats of a short bench.py run (no counters). Summarise with
# `python tools/prof_summary.py gpurun_out/prof_<tag>`.
# usage: tools/prof_step.sh <tag> [bench.py args...]
set -e
tag=$1; shift
repo=$(pwd)
out=$repo/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run \
  -- python3 "$repo/bench.py" "$@" > "$out.log" 2>&1
