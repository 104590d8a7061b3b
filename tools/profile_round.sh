#!/bin/bash
# rocprofv3 evidence for bench.py, run on the GPU box from the repo root:
#   bash tools/profile_round.sh <tag> [bench args...]
# 1) kernel trace + stats of the bench command (no PMC); 2) FETCH_SIZE pass; 3) WRITE_SIZE pass;
# 4) SQ/GRBM pass (MFMA busy cycles, wave states) — separate --pmc runs, no tracing domains.
# Outputs under gpurun_out/prof_<tag>/, plus traffic.json (per kernel instance, stamped with the
# kernel sources' hash and the workload).
set -e
TAG=${1:-r02}
shift || true
EXTRA="$*"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile --no-secondary --sustain 0 $EXTRA"
WL=$(python3 bench.py --print-workload $EXTRA)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
python3 tools/pmc_traffic.py "$WL" $OUT/traffic.json $(find $OUT/fetch -name '*counter_collection.csv' | head -1) $(find $OUT/write -name '*counter_collection.csv' | head -1) $(find $OUT/sq -name '*counter_collection.csv' | head -1) $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 5
python3 tools/gap_summary.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 5 > $OUT/trace_summary.txt
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
echo profile-done
