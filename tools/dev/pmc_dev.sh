#!/bin/bash
# Development PMC pass for kernels matching a regex (run on the GPU box from the repo root):
#   bash tools/pmc_dev.sh <tag> <kernel-regex> "<counters>"
export TMPDIR=/tmp
TAG=$1; RE=$2; CTRS=$3
OUT=gpurun_out/pmc_$TAG
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc $CTRS --kernel-include-regex "$RE" --output-format csv -d $OUT -o run -- python3 bench.py --steps 2 --warmup 2 --cpu-steps 0 --no-mse --no-profile > $OUT/log 2>&1
f=$(find $OUT -name '*counter_collection.csv' | head -1)
cp $f $OUT/cc.csv
