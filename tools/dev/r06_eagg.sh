#!/bin/bash
# Round 6: edge-side aggregation — GPU tests, then Cfg E (aneurysm) A/B (MGN_EDGE_AGG=0 vs auto) on one box.
#   bash tools/dev/r06_eagg.sh <tag> [skip-tests]
TAG=${1:-r06e}
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_edge_agg_gpu.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/eagg_tests_$TAG.log 2>&1
  rc=$?; echo tests=$rc; grep -E "passed|failed|worst|Error" gpurun_out/eagg_tests_$TAG.log | tail -12
  [ $rc -eq 0 ] || exit $rc
fi
for mode in 0 auto 0 auto; do
  MGN_EDGE_AGG=$mode timeout -k 10 300 python bench.py --workload aneurysm --steps 10 --warmup 3 --cpu-steps 0 --no-secondary --no-mse > gpurun_out/eagg_${TAG}_$mode.json 2> gpurun_out/eagg_${TAG}_$mode.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/eagg_${TAG}_$mode.json'))
k=d['kernels']; print('$mode', d['value'], d['ms_per_step'], ' '.join('%s=%.1f' % (c, k[c]['avg_us']) for c in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad') if c in k))"
done
