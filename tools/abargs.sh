#!/bin/bash
# Interleaved A/B/... of bench.py on ONE box: each arm is "ENV=.. ENV2=.. :: bench args" (either
# part optional).  Usage: tools/abargs.sh ROUNDS "ARM_A" "ARM_B" ["ARM_C" ...]
R=$1; shift
run_arm() {
  local spec="$1" envs="" args=""
  if [[ "$spec" == *"::"* ]]; then envs="${spec%%::*}"; args="${spec#*::}"; else args="$spec"; fi
  out=$(env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $args 2>/dev/null | tail -1) || { echo "fail [$spec]"; exit 1; }
  echo "[$spec] $(echo "$out" | python3 -c 'import json,sys; print(json.load(sys.stdin)["ms_per_step"])')"
}
for i in $(seq 1 "$R"); do
  for arm in "$@"; do run_arm "$arm" || exit 1; done
done
