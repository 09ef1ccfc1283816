#!/bin/bash
# Usage (GPU box, repo root): tools/pmc.sh NAME "COUNTERS" -- python3 script.py args...
# rocprofv3 hardware-counter run (kernel trace + --pmc only; no sys/runtime traces), summary
# per kernel via tools/pmc_summary.py into gpurun_out/pmc_NAME/summary.md.
set -o pipefail
name=$1; shift; counters=$1; shift; [ "$1" == "--" ] && shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/pmc_$name
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
rocprofv3 --kernel-trace --pmc $counters -f csv -d "$out" -o run -- "$@"
rc=$?
f=$(find "$out" -name '*counter_collection.csv' | head -1)
if [ -n "$f" ]; then
  python3 "$root/tools/pmc_summary.py" "$f" > "$out/summary.md" 2>&1 || true
  find "$out" -name '*counter_collection.csv' -size +20M -delete
fi
find "$out" -name '*kernel_trace.csv' -size +20M -delete
exit $rc
