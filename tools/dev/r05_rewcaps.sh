#!/bin/bash
# Round 5: Cfg B with the recomputed weight gradients under other concurrent-backward CU splits
set -o pipefail
row() {  # tag env bench-args
  env $2 timeout -k 10 300 python bench.py $3 > gpurun_out/rc_$1.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/rc_$1.log; exit 1; }
  echo $1 $(tail -1 gpurun_out/rc_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
}
B="--steps 40 --warmup 5 --cpu-steps 0 --no-mse --sustain 0 --no-secondary --no-profile"
row base "MGN_REW=0" "$B"
for c in 160,96 128,128 112,144 96,160; do row rew_$c "MGN_REW=1 MGN_CONC_WGRAD=$c" "$B"; done
row base2 "MGN_REW=0" "$B"
