#!/bin/bash
# usage: envab.sh ROUNDS "ENV_A" "ENV_B" [bench args]: alternate bench runs with two env settings
R=$1; A=$2; B=$3; shift 3
for i in $(seq 1 $R); do
  for arm in "$A" "$B"; do
    out=$(env $arm timeout -k 10 200 python bench.py --steps 20 --warmup 5 "$@" 2>/dev/null | tail -1) || { echo "fail $arm"; exit 1; }
    echo "$arm $(echo "$out" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
  done
done
