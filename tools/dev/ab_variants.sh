#!/bin/bash
# Diagnostics on the GPU box: bench each relinked variant (tools/build_variant.sh) against the default
# library; per-class kernel times. bash tools/ab_variants.sh v1 v2 ...
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
for v in default "$@"; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 0 > gpurun_out/var_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var_$v.log; cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
  echo $v $(tail -1 gpurun_out/var_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','fwd_node','bwd_node','combine','wgrad','proj','fwd_dense','bwd_dense') if n in k))")
done
cp /tmp/libmgn_default.so $L/libmgn.so
