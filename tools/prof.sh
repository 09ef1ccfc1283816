#!/bin/bash
# Usage (on the GPU box, from the repo root): tools/prof.sh NAME -- python3 script.py args...
# Runs rocprofv3 kernel-trace+stats (CSV) and keeps only the small summary files under
# gpurun_out/prof_NAME (the per-dispatch trace is deleted to stay under gpurun's copy-back cap).
set -o pipefail
name=$1; shift; [ "$1" == "--" ] && shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof_$name
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
rocprofv3 --kernel-trace --stats -f csv -T -d "$out" -o run -- "$@"
rc=$?
find "$out" -name '*kernel_trace.csv' -size +2M -delete
find "$out" -name '*.db' -delete
exit $rc
