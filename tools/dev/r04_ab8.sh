#!/bin/bash
# small graphs (Cfg A fp32 h=32, Cfg C plate bf16 h=64): the concurrent backward with one workspace per
# block (no lock-step waits on the main stream) and uncapped / split grids, against one stream
TAG=${1:-ab8}
run() {  # run <label> <bench args> -- <env...>
  local lab=$1; shift
  local args=()
  while [ "$1" != "--" ]; do args+=("$1"); shift; done; shift
  env "$@" timeout -k 10 200 python bench.py --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2 \
    "${args[@]}" > gpurun_out/ab_${TAG}_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/ab_${TAG}_$lab.log; return 1; }
  echo "$lab $(tail -1 gpurun_out/ab_${TAG}_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], (d.get('sustained') or {}).get('value'))")"
}
A="--mp 5 --hidden 32 --batch 1 --dtype fp32"
C="--workload plate --mp 10 --hidden 64 --batch 1 --dtype bf16"
run a_one $A -- MGN_CONC_WGRAD=0 && run a_u2 $A -- MGN_CONC_WGRAD=0,0 && run a_uall $A -- MGN_CONC_WGRAD=0,0 MGN_CONC_WS=all \
  && run a_s_all $A -- MGN_CONC_WGRAD=160,96 MGN_CONC_WS=all && run a_one_b $A -- MGN_CONC_WGRAD=0 \
  && run c_one $C -- MGN_CONC_WGRAD=0 && run c_uall $C -- MGN_CONC_WGRAD=0,0 MGN_CONC_WS=all \
  && run c_s_all $C -- MGN_CONC_WGRAD=160,96 MGN_CONC_WS=all && run c_one_b $C -- MGN_CONC_WGRAD=0
