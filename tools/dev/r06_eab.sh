#!/bin/bash
# Round 6: edge-side aggregation ablation at Cfg E (variant builds of mgn_chain16.hip, tools/build_variant.sh;
# diagnostics only: the ablated variants compute wrong aggregates). Rows: variant, MGN_EDGE_AGG, steps/s,
# ms/step, per-class avg us.   bash tools/dev/r06_eab.sh <tag> <variants...>
TAG=$1; shift
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
row() {  # variant mode
  MGN_EDGE_AGG=$2 timeout -k 10 300 python bench.py --workload aneurysm --steps 10 --warmup 3 --cpu-steps 0 --no-secondary --no-mse --sustain 0 > gpurun_out/eab_${TAG}_$1_$2.json 2> gpurun_out/eab_${TAG}_$1_$2.err || return 1
  python3 -c "
import json; d=json.load(open('gpurun_out/eab_${TAG}_$1_$2.json'))
k=d['kernels']; print('$1', '$2', d['value'], d['ms_per_step'], ' '.join('%s=%.1f' % (c, k[c]['avg_us']) for c in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad') if c in k))"
}
row default 0 || exit 1
for v in default "$@"; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  row $v auto || { cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
done
cp /tmp/libmgn_default.so $L/libmgn.so
