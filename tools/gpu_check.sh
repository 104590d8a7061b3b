#!/bin/bash
# GPU tests + short bench (development; run on the GPU box from the repo root): bash tools/gpu_check.sh <tag> [pytest -k expr]
TAG=${1:-dev}
K=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2; grep -E "^E  " gpurun_out/gpu_tests_$TAG.log | head -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/bench_$TAG.log 2>&1
echo bench=$?
tail -1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['one_step_mse']['abs_diff']); print(json.dumps(d['roofline'])[:600]); [print(k, v) for k, v in d['kernels'].items()]" || tail -5 gpurun_out/bench_$TAG.log
