#!/bin/bash
# Round 6: the timed-step count's effect on the Cfg B line (same box): K/W = 20/5 (old default) vs 100/20.
mkdir -p gpurun_out
for kw in "20 5" "100 20" "20 5" "100 20"; do
  set -- $kw
  timeout -k 10 300 python bench.py --steps $1 --warmup $2 --cpu-steps 0 --no-secondary --no-mse --no-profile > gpurun_out/steps_$1_$2.json 2> gpurun_out/steps_$1_$2.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/steps_$1_$2.json')); print('K=$1 W=$2', d['value'], d['ms_per_step'], d['sustained']['value'])"
done
