#!/bin/bash
# Run GPU steps on the gpurun box with per-step time limits.
#   tools/gpu_steps.sh "name:timeout:cmd" ...
# A step that exits 0 or 1 (ordinary failure, e.g. failing asserts) lets the
# next step run; any other status (abort, segfault, timeout, GPU fault) ends
# the script there.
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; to=${rest%%:*}; cmd=${rest#*:}
  echo "=== [$name] (limit ${to}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "=== stopping after [$name]"; exit $rc; fi
done
