#!/bin/bash
# rocprofv3 kernel traces of the headline step, one stream vs MGN_CONC_WGRAD splits.
#   bash tools/dev/prof_conc.sh <tag> "160,96" ...
TAG=$1; shift
export TMPDIR=/tmp
B="--steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile --no-secondary --sustain 0"
for v in 0 "$@"; do
  OUT=gpurun_out/profc_${TAG}_${v/,/_}
  mkdir -p $OUT
  MGN_CONC_WGRAD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $B > $OUT/trace.log 2>&1 || exit 1
  python3 tools/gap_summary.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 5 > $OUT/trace_summary.txt
  echo "== $v"; head -12 $OUT/trace_summary.txt
done
