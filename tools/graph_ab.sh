#!/bin/bash
# hipGraph execution-mode A/B (eager vs graph replay under HIP runtime graph knobs), 20 timed
# steps each, R rounds interleaved.  Usage: tools/graph_ab.sh R
R=${1:-2}
for i in $(seq 1 $R); do
  for arm in "eager::--no-graph" "graph::--graph" "q2:DEBUG_HIP_FORCE_GRAPH_QUEUES=2:--graph" \
             "q4:DEBUG_HIP_FORCE_GRAPH_QUEUES=4:--graph" "pkt:DEBUG_CLR_GRAPH_PACKET_CAPTURE=1:--graph"; do
    name=${arm%%:*}; rest=${arm#*:}; envs=${rest%%:*}; flags=${rest#*:}
    out=$(env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 $flags 2>/dev/null | tail -1) \
      || { echo "fail $name"; exit 1; }
    echo "$name $(echo "$out" | python3 -c 'import json,sys; j=json.load(sys.stdin); print(j["ms_per_step"], j["config"]["hip_graph"])')"
  done
done
