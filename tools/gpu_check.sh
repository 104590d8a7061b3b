#!/bin/bash
# GPU tests + short bench (used during development; run on the GPU box from the repo root)
TAG=${1:-dev}
timeout -k 10 500 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
echo tests=$?; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2; grep -E "^E  " gpurun_out/gpu_tests_$TAG.log | head -4
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/bench_$TAG.log 2>&1
echo bench=$?
tail -1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['one_step_mse']['abs_diff']); [print(k, v['avg_us'], round(v['total_ms']/d['steps'],3)) for k, v in d['kernels'].items()]" || tail -5 gpurun_out/bench_$TAG.log
