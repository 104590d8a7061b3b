#!/bin/bash
# Round 5: kernel-argument placement (HIP_FORCE_DEV_KERNARG) on the small graphs, same library
set -o pipefail
i=0
for e in "" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" ""; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2 > gpurun_out/karg_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/karg_$i.log; exit 1; }
  echo "[$e]" $(tail -1 gpurun_out/karg_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','wgrad') if n in k))")
done
