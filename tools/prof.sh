#!/bin/bash
# Usage (on the GPU box, from the repo root): tools/prof.sh NAME -- python3 script.py args...
# Runs rocprofv3 kernel-trace+stats (CSV) under gpurun_out/prof_NAME, writes a per-step summary
# (tools/trace_summary.py) next to it and drops the per-dispatch trace if it is large.
set -o pipefail
name=$1; shift; [ "$1" == "--" ] && shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof_$name
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
rocprofv3 --kernel-trace --stats -f csv -T -d "$out" -o run -- "$@"
rc=$?
if [ -f "$out/run_kernel_trace.csv" ]; then
  python3 "$root/tools/trace_summary.py" "$out/run_kernel_trace.csv" --steps ${PROF_STEPS:-5} --list \
    > "$out/summary.md" 2>&1 || true
fi
find "$out" -name '*kernel_trace.csv' -size +20M -delete
find "$out" -name '*.db' -delete
exit $rc
