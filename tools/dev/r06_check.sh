#!/bin/bash
# Round 6 development check (GPU box, repo root): GPU tests (optionally -k), the default bench line, and
# bench.py's own N-rank launcher rehearsed with 2 gloo ranks sharing the GPU.
#   bash tools/dev/r06_check.sh <tag> [pytest -k expr] [skip-tests]
TAG=${1:-r06}
K=${2:-}
mkdir -p gpurun_out
if [ -z "$3" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?
  echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2; grep -E "^E  " gpurun_out/gpu_tests_$TAG.log | head -8
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench=$?
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print(d['value'], d['ms_per_step'], d.get('sustained'), d['one_step_mse']['abs_diff'])
print(json.dumps(d['roofline'])[:500])
for k, v in d['kernels'].items(): print(k, v)
for k, v in d.get('secondary', {}).items(): print(k, v['value'], v['ms_per_step'])
" || exit 1
MGN_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-profile --sustain 1 --cpu-steps 0 --no-secondary > gpurun_out/launch2_$TAG.json 2> gpurun_out/launch2_$TAG.err
echo launch2=$?
cat gpurun_out/launch2_$TAG.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['config']['parallelism'], d['value'], d['optimizer_steps_per_s'], d.get('data_parallel'))"
