#!/bin/bash
# Development check on the GPU box: full GPU suite (minus -k exclusions) + short bench.
# bash tools/dev_check.sh <tag> [pytest -k expr]
TAG=${1:-dev}
K=${2:-}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s -p no:cacheprovider --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/dev_tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|one-step MSE" gpurun_out/dev_tests_$TAG.log | tail -4; grep -E "^E  " gpurun_out/dev_tests_$TAG.log | head -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse > gpurun_out/dev_bench_$TAG.log 2>&1
echo bench=$?
tail -1 gpurun_out/dev_bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v['avg_us'], v['ms_per_step']) for k, v in d['kernels'].items()]" || tail -5 gpurun_out/dev_bench_$TAG.log
