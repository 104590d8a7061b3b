#!/bin/bash
# Small-graph rows (Cfg A, Cfg C at plate.json's sizes) for each relinked variant
# (tools/build_variant.sh) against the default library. bash tools/dev/small_variants.sh <tag> v1 v2 ...
TAG=$1; shift
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
for v in default "$@"; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  for w in "A:--dtype fp32 --mp 5 --hidden 32 --batch 1" "C:--workload plate --mp 10 --hidden 64 --batch 1"; do
    t=${w%%:*}; args=${w#*:}
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-steps 0 --no-mse --no-secondary --sustain 2 $args > gpurun_out/smv_${TAG}_${v}_$t.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/smv_${TAG}_${v}_$t.log; cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
    echo "$v $t $(tail -1 gpurun_out/smv_${TAG}_${v}_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], (d.get('sustained') or {}).get('value'), ' '.join('%s=%s' % (n, v['avg_us']) for n, v in k.items() if n in ('wgrad','wgrad_dense','wgrad_reduce','fwd_edge','fwd_node','bwd_edge','bwd_node')))")"
  done
done
cp /tmp/libmgn_default.so $L/libmgn.so
