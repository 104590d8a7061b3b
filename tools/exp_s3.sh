#!/bin/bash
# dev: GPU tests + Cfg B bench + Cfg E (aneurysm) bench kernel times
bash tools/gpu_check.sh ${1:-s3} || exit 1
timeout -k 10 300 python3 bench.py --workload aneurysm --steps 5 --warmup 2 --cpu-steps 0 --no-mse > gpurun_out/bench_an_${1:-s3}.log 2>&1
echo an=$?
tail -1 gpurun_out/bench_an_${1:-s3}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']); [print(k, v['avg_us'], round(v['total_ms']/d['steps'],3)) for k, v in d['kernels'].items()]"
