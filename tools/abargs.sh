#!/bin/bash
# Interleaved A/B of bench.py on ONE box: each arm is "ENV=.. ENV2=.. :: bench args" (either part
# optional).  Usage: tools/abargs.sh ROUNDS "ARM_A" "ARM_B"
R=$1; A=$2; B=$3
run_arm() {
  local spec="$1" envs="" args=""
  if [[ "$spec" == *"::"* ]]; then envs="${spec%%::*}"; args="${spec#*::}"; else args="$spec"; fi
  out=$(env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $args 2>/dev/null | tail -1) || { echo "fail [$spec]"; exit 1; }
  echo "[$spec] $(echo "$out" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
}
for i in $(seq 1 "$R"); do run_arm "$A"; run_arm "$B"; done
