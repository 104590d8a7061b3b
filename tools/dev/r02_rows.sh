#!/bin/bash
# Round-2 secondary rows on the GPU box: new parity tests (trained-model MSE, reference rollout
# fixture, 2-rank libmgn DP), then fp32 Cfg B and the eager fresh-batch (Lightning-path) step.
# bash tools/r02_rows.sh <tag>
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_trained_gpu.py tests/test_rollout_gpu.py tests/test_distributed_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/rows_tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|one-step MSE" gpurun_out/rows_tests_$TAG.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse > gpurun_out/bench_fp32_$TAG.log 2>&1
rc=$?; echo fp32=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --fresh-batch --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-profile > gpurun_out/bench_fresh_$TAG.log 2>&1
rc=$?; echo fresh=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-graph --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-profile > gpurun_out/bench_eager_$TAG.log 2>&1
rc=$?; echo eager=$rc; [ $rc -eq 0 ] || exit $rc
for f in fp32 fresh eager; do tail -1 gpurun_out/bench_${f}_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['dtype'], d['execution'][:60])"; done
