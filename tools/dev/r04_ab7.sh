#!/bin/bash
# decoder weight gradients beside the last block's data half (MGN_DEC_SPLIT) + the parity tests they touch
TAG=${1:-ab7}
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_step_gpu.py tests/test_abi.py > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/ab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # run <label> <env...>
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3 \
    > gpurun_out/ab_${TAG}_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/ab_${TAG}_$lab.log; return 1; }
  echo "$lab $(tail -1 gpurun_out/ab_${TAG}_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], (d.get('sustained') or {}).get('value'))")"
}
run dec1 MGN_DEC_SPLIT=1 && run dec0 MGN_DEC_SPLIT=0 && run dec1b MGN_DEC_SPLIT=1 && run dec0b MGN_DEC_SPLIT=0
