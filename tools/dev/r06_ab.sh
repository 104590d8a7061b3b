#!/bin/bash
# Round 6: same-box A/B of variant libraries on one workload (bench.py per-class times).
#   bash tools/dev/r06_ab.sh <tag> "<bench args>" <variant>...
TAG=$1; ARGS=$2; shift 2
L=graph-physics_amd/graphphysics/_lib
mkdir -p gpurun_out
cp $L/libmgn.so /tmp/libmgn_default.so
for v in default "$@" default "$@"; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  timeout -k 10 300 python bench.py $ARGS --steps 10 --warmup 3 --cpu-steps 0 --no-secondary --no-mse --sustain 0 > gpurun_out/ab_${TAG}_$v.json 2> gpurun_out/ab_${TAG}_$v.err || { cp /tmp/libmgn_default.so $L/libmgn.so; tail -5 gpurun_out/ab_${TAG}_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_${TAG}_$v.json'))
k=d['kernels']; print('$v', d['value'], d['ms_per_step'], ' '.join('%s=%.1f' % (c, k[c]['avg_us']) for c in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad','fwd_dense','bwd_dense') if c in k))"
done
cp /tmp/libmgn_default.so $L/libmgn.so
