#!/bin/bash
# Round 5 A/B on one box: bench.py rows for the default library and relinked variants
# (tools/build_variant.sh). bash tools/dev/r05_ab.sh "<bench args>" tag v1 v2 ...
ARGS=$1; TAG=$2; shift 2
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
for v in default "$@" default; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  timeout -k 10 300 python bench.py $ARGS > gpurun_out/ab_${TAG}_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/ab_${TAG}_$v.log; cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
  echo $TAG $v $(tail -1 gpurun_out/ab_${TAG}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], (d.get('sustained') or {}).get('value'), ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','fwd_node','bwd_node','combine','wgrad','proj','fwd_dense','bwd_dense') if n in k))")
done
cp /tmp/libmgn_default.so $L/libmgn.so
