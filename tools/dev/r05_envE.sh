#!/bin/bash
# Round 5: concurrent backward at Cfg E (recomputed weight gradients on), environment only
TAG=$1; shift
i=0
for e in "" "$@" ""; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --workload aneurysm --batch 1 --steps 10 --warmup 2 --cpu-steps 0 --no-mse --no-secondary --no-profile --sustain 0 > gpurun_out/envE_${TAG}_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/envE_${TAG}_$i.log; exit 1; }
  echo "[$e]" $(tail -1 gpurun_out/envE_${TAG}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
done
