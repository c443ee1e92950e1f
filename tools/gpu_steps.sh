#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that ends in a fault,
# abort, segfault, signal or time limit (exit >= 124), keep going after ordinary failures (exit 1-2:
# a failed assertion).  Usage: tools/gpu_steps.sh "<seconds> <name> <command...>" ...
# Output of step <name> goes to gpurun_out/<name>.log.
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  secs=${spec%% *}; rest=${spec#* }
  name=${rest%% *}; cmd=${rest#* }
  echo "=== [$name] $cmd (limit ${secs}s) $(date +%T)"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc $(date +%T)"
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then
    echo "=== stopping: step $name ended with $rc"
    exit $rc
  fi
done
exit 0
