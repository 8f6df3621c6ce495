#!/bin/bash
# Runs GPU steps in sequence on a gpurun box; stops at the first step that ends abnormally
# (GPU fault / abort / segfault / timeout). Plain test failures (rc 1) do not stop the chain.
# usage: tools/gpu_session.sh "name:timeout:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "[gpu_session] >>> $name (timeout ${tmo}s): $cmd"
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_session] <<< $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[gpu_session] abnormal exit ($rc), stopping"; exit $rc
  fi
done
