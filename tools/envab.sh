#!/bin/bash
# usage: envab.sh ROUNDS "ENV_A" "ENV_B" ["ENV_C" ...] [-- bench args]
# Interleaved bench runs of every env arm per round (one box, same build); prints ms/step.
R=$1; shift
arms=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do arms+=("$1"); shift; done
[ "$1" == "--" ] && shift
for i in $(seq 1 $R); do
  for arm in "${arms[@]}"; do
    out=$(env $arm timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" 2>/dev/null | tail -1) || { echo "fail $arm"; exit 1; }
    echo "$arm $(echo "$out" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
