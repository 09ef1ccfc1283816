#!/bin/bash
# A/B of the step time on ONE box: ab/base (a git worktree of the baseline commit with its own
# in-tree build) against the working tree, interleaved R rounds (box-to-box clock variance is
# larger than most single changes).  Usage (GPU box, repo root): tools/ab.sh [ROUNDS] [bench args]
set -o pipefail
R=${1:-3}; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
for i in $(seq 1 "$R"); do
  for arm in base new; do
    if [ $arm == base ]; then dir=$root/ab/base; else dir=$root; fi
    out=$( cd "$dir" && timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" 2>/dev/null | tail -1 )
    rc=$?
    [ $rc -ne 0 ] && { echo "$arm failed rc=$rc"; exit $rc; }
    echo "$arm $(echo "$out" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
