#!/bin/bash
# Batch-size scaling of the step and per-kernel durations (fixed vs per-edge cost), GPU box, repo root.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/scal
mkdir -p $OUT
for B in 4 8 16 32; do
  timeout -k 10 200 python3 bench.py --batch $B --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-profile > $OUT/b$B.log 2>&1
  echo B=$B $(tail -1 $OUT/b$B.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
done
for B in 8 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr$B -o run -- python3 bench.py --batch $B --steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile > $OUT/tr$B.log 2>&1
  python3 tools/gap_summary.py $OUT/tr$B/run_kernel_trace.csv 5 > $OUT/gaps$B.txt
done
echo done
