#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop the whole call on a fault-class
# exit (abort 134, segfault 139, timeout 124/137, signal-negative) — never retry a GPU step.
# usage: tools/gpu_steps.sh "name:seconds:command" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|5) ;;                       # ok / pytest test failures / no tests collected
    *) echo "=== stopping: fault-class exit $rc in $name"; exit $rc ;;
  esac
done
