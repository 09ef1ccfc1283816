set -o pipefail
for i in 1 2; do
for arm in "eager::--no-graph" "graph::--graph" "graph_nowg:SIMCLR_WGRAD_STREAM=0:--graph" "graph_1s:SIMCLR_WGRAD_STREAM=0 SIMCLR_BRANCH_STREAM=0:--graph" "eager_1s:SIMCLR_WGRAD_STREAM=0 SIMCLR_BRANCH_STREAM=0:--no-graph"; do
  name=${arm%%:*}; rest=${arm#*:}; envs=${rest%%:*}; flags=${rest#*:}
  out=$(env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $flags 2>/dev/null | tail -1) || { echo "fail $name"; exit 1; }
  echo "$name $(echo "$out" | python3 -c 'import json,sys; j=json.load(sys.stdin); print(j["ms_per_step"], j["config"]["hip_graph"])')" >> gpurun_out/graph21.txt
done
done
