#!/bin/bash
TAG=${1:-ab6}
run() {  # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3 \
    > gpurun_out/ab_${TAG}_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/ab_${TAG}_$lab.log; return 1; }
  echo "$lab $(tail -1 gpurun_out/ab_${TAG}_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], (d.get('sustained') or {}).get('value'))")"
}
run enc1 MGN_ENC_CAP=1 && run enc0 MGN_ENC_CAP=0 && run enc1b MGN_ENC_CAP=1 && run enc0b MGN_ENC_CAP=0
