#!/bin/bash
# fp32 Cfg B step: default library vs relinked variants (tools/build_variant.sh), per-class kernel times.
# bash tools/ab_fp32.sh v1 v2 ...
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
for v in default "$@"; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  timeout -k 10 200 python bench.py --dtype fp32 --steps 10 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 0 > gpurun_out/var32_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var32_$v.log; cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
  echo $v $(tail -1 gpurun_out/var32_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in k))")
done
cp /tmp/libmgn_default.so $L/libmgn.so
