#!/bin/bash
# Round 5: concurrent-backward schedule knobs (environment only, same library), bf16 Cfg B, one box.
# bash tools/dev/r05_env.sh tag "ENV=.. ENV2=.." "..." ...
TAG=$1; shift
i=0
for e in "" "$@" ""; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --no-profile --sustain 3 > gpurun_out/env_${TAG}_$i.log 2>&1 || { echo "[$e] failed"; tail -3 gpurun_out/env_${TAG}_$i.log; exit 1; }
  echo "[$e]" $(tail -1 gpurun_out/env_${TAG}_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['sustained']['value'])")
done
