#!/bin/bash
# Acquire a GPU box for one command, retrying ONLY while gpurun exits 3 (no box / slot free: nothing
# ran, nothing charged). Any other outcome (the command ran, failed, timed out, refused) ends the loop.
#   bash tools/gpu_retry.sh <timeout_s> <out_file> '<command>'
T=$1; OUT=$2; CMD=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$CMD" > $OUT 2>&1
  rc=$?
  [ $rc -eq 3 ] || exit $rc
  sleep 45
done
exit 3
