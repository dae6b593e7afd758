#!/bin/bash
# Run GPU steps in order; each under its own time limit; stop at the first crash-type exit
# (fault/abort/segfault/timeout) so nothing else touches the GPU after it.
# usage: tools/gpu_steps.sh "<secs>|<name>|<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"; tail -5 "gpurun_out/$name.log"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] || [ $rc -gt 128 ]; then
    echo "=== stopping after crash-type exit $rc"; exit $rc
  fi
done
