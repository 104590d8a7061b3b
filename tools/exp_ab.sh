#!/bin/bash
# dev A/B: GPU tests + bench on libmgn.so (A), then bench on an alternate build (B) copied over it
# bash tools/exp_ab.sh <tag> <alt .so path>
set -o pipefail
TAG=${1:-ab}
bash tools/gpu_check.sh ${TAG}A || exit 1
grep -q "failed" gpurun_out/gpu_tests_${TAG}A.log && exit 1
[ -n "$2" ] || exit 0
cp "$2" graph-physics_amd/graphphysics/_lib/libmgn.so
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/bench_${TAG}B.log 2>&1
echo benchB=$?
tail -1 gpurun_out/bench_${TAG}B.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['one_step_mse']['abs_diff']); [print(k, v['avg_us'], round(v['total_ms']/d['steps'],3)) for k, v in d['kernels'].items()]"
