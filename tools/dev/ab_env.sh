#!/bin/bash
# Diagnostics on the GPU box: bench the default library under alternating environment settings
# (switches that do not change results). bash tools/ab_env.sh "MGN_PAIR_DE=0" "MGN_PAIR_DE=1" ...
for e in "$@"; do
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse > gpurun_out/env_ab.log 2>&1 || { echo "$e failed"; tail -3 gpurun_out/env_ab.log; exit 1; }
  echo "$e" $(tail -1 gpurun_out/env_ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','fwd_node','bwd_node','combine','wgrad','fwd_dense','bwd_dense') if n in k))")
done
