#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root).
# 1) kernel trace + stats; 2) FETCH_SIZE pass; 3) WRITE_SIZE pass (separate --pmc runs, no tracing domains)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p $OUT
ARGS="--steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo done
