#!/bin/bash
# per-kernel-class times at batch 1, 2, 4, 8 (fixed vs per-graph cost of each class)
for B in 1 2 4 8; do
  timeout -k 10 200 python bench.py --batch $B --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 0 > gpurun_out/sweep_b$B.log 2>&1 || exit 1
  echo B=$B $(tail -1 gpurun_out/sweep_b$B.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['ms_per_step'], ' '.join('%s=%.1f/%d' % (n, 1000*k[n]['ms_per_step'], k[n]['launches']//20) for n in sorted(k)))")
done
