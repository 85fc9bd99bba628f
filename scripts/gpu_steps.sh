#!/bin/bash
# Run GPU steps in order; each step has its own time limit.  A step that fails normally (exit 1:
# test failures) lets the next step run; a fault / abort / segfault / time limit ends the call.
#   scripts/gpu_steps.sh "<secs>:<name>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  secs=${spec%%:*}
  rest=${spec#*:}
  name=${rest%%:*}
  cmd=${rest#*:}
  echo "=== [$name] $cmd (limit ${secs}s)"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping after [$name] (exit $rc)"; exit $rc ;;
  esac
done
