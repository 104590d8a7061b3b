#!/bin/bash
# concurrent backward workspaces: one per block (MGN_CONC_WS=all) vs two alternating, same box
TAG=${1:-ab4}
run() {  # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3 \
    > gpurun_out/ab_${TAG}_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/ab_${TAG}_$lab.log; return 1; }
  echo "$lab $(tail -1 gpurun_out/ab_${TAG}_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], (d.get('sustained') or {}).get('value'))")"
}
run ws_2 MGN_CONC_WS=2 && run ws_3 MGN_CONC_WS=3 && run ws_2_sr MGN_CONC_WS=2 MGN_SIDE_REDUCE=1 && run ws_3_sr MGN_CONC_WS=3 MGN_SIDE_REDUCE=1 && \
  run ws_2b MGN_CONC_WS=2 && run ws_3b MGN_CONC_WS=3 || exit 1
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "concurrent_weight_gradients or captured_step_equals_eager" > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/ab_tests_$TAG.log; exit $rc
