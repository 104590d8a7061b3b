#!/bin/bash
# Whole GPU suite without -x (every failure listed) + default bench line (development; run on the
# GPU box from the repo root): bash tools/gpu_full.sh <tag> [pytest -k expr]
TAG=${1:-dev}
K=${2:-}
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests_$TAG.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1
echo bench=$?
tail -1 gpurun_out/bench_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('sustained'), d['one_step_mse']['abs_diff'], d.get('cpu_baseline')); print(json.dumps(d['roofline'])[:700]); print(json.dumps(d.get('secondary'))[:3000])" || tail -5 gpurun_out/bench_$TAG.log
