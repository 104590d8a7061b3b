#!/bin/bash
# Round 6: edge-side aggregation forced on at Cfg B (MGN_EDGE_AGG=1 vs 0), A/B on one box
TAG=${1:-r06b}
mkdir -p gpurun_out
for mode in 0 1 0 1; do
  MGN_EDGE_AGG=$mode timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-secondary --no-mse > gpurun_out/eaggB_${TAG}_$mode.json 2> gpurun_out/eaggB_${TAG}_$mode.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/eaggB_${TAG}_$mode.json'))
k=d['kernels']; print('$mode', d['value'], d['ms_per_step'], d['sustained']['value'], ' '.join('%s=%.1f' % (c, k[c]['avg_us']) for c in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad') if c in k))"
done
