#!/bin/bash
# rocprofv3 evidence for bench.py, run on the GPU box from the repo root:
#   bash tools/profile_round.sh r01
# 1) kernel trace + stats (the same bench command, no PMC); 2) FETCH_SIZE pass; 3) WRITE_SIZE pass
# (separate --pmc runs, no tracing domains). Outputs under gpurun_out/prof_<tag>/ plus
# gpurun_out/prof_<tag>/traffic.json (bytes per launch per kernel class, source-hash stamped).
set -e
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv $OUT/traffic.json
echo profile-done
