#!/bin/bash
# Run a list of GPU steps on the gpurun box, each under its own time limit, stopping at the
# first step that faults / aborts / times out (exit >= 124).  Test failures (exit 1) continue.
# Usage: tools/gpu_steps.sh "NAME|SECONDS|COMMAND" ...
out=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "=== [$name] ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "$out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping after fatal rc=$rc in $name"
    exit $rc
  fi
done
exit 0
