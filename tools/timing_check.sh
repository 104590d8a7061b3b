#!/bin/bash
# Diagnostics on the GPU box: bench.py's per-kernel averages (profiled eager steps) next to the
# rocprofv3 kernel trace of the replayed steps, on the same box. bash tools/timing_check.sh <tag>
set -e
TAG=${1:-tc}
export TMPDIR=/tmp
OUT=gpurun_out/tc_$TAG
mkdir -p $OUT
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse > $OUT/bench.log 2>&1
tail -1 $OUT/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in k))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile > $OUT/trace.log 2>&1
python3 tools/gap_summary.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 5 
