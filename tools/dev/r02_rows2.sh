#!/bin/bash
# Round-2 secondary rows with rocprofv3 kernel statistics (run on the GPU box from the repo root):
# Cfg C plate and Cfg E aneurysm training steps, fp32 Cfg B, eager fresh-batch (Lightning-path) Cfg B.
# bash tools/r02_rows2.sh <tag>
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > gpurun_out/${TAG}_bench_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/${TAG}_bench_$n.log; return 1; }
  tail -1 gpurun_out/${TAG}_bench_$n.log > gpurun_out/${TAG}_bench_$n.json
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$n.json')); print('$n', d['value'], d['ms_per_step'], d['config']['workload'][:50])"
}
prof() {  # name, bench args: rocprofv3 kernel trace + stats of a short run
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$n -o run -- python3 bench.py "$@" > gpurun_out/${TAG}_prof_$n.log 2>&1 || { echo "prof $n failed"; return 1; }
  cp $(find gpurun_out/${TAG}_prof_$n -name '*kernel_stats.csv' | head -1) gpurun_out/${TAG}_kernel_stats_$n.csv
  echo "prof $n ok"
}
run plate --workload plate --steps 20 --warmup 3 --cpu-steps 0 || exit 1
run aneurysm --workload aneurysm --steps 10 --warmup 2 --cpu-steps 0 --no-mse || exit 1
run fp32 --dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse || exit 1
run fresh --fresh-batch --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-profile || exit 1
prof fp32 --dtype fp32 --steps 5 --warmup 2 --cpu-steps 0 --no-mse --no-profile || exit 1
prof fresh --fresh-batch --steps 5 --warmup 2 --cpu-steps 0 --no-mse --no-profile || exit 1
prof plate --workload plate --steps 5 --warmup 2 --cpu-steps 0 --no-mse --no-profile || exit 1
echo rows-done
