#!/bin/bash
# Kernel-trace a short bench run per mode and summarise GPU idle (tools/idle_summary.py):
#   tools/runidle.sh NAME [bench args...]
set -o pipefail
name=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/idle_$name
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -f csv -d "$out" -o run -- python3 "$root/bench.py" --steps 8 --warmup 3 "$@" > "$out/bench.json"
rc=$?
python3 "$root/tools/idle_summary.py" "$out/run_kernel_trace.csv" 5 > "$out/idle.txt" 2>&1
find "$out" -name '*.csv' -size +30M -delete
exit $rc
