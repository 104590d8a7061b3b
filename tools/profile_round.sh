#!/bin/bash
# rocprofv3 evidence for bench.py, run on the GPU box from the repo root:
#   bash tools/profile_round.sh <tag> [bench args...]
# 1) kernel trace + stats of the bench command (no PMC; the default schedule: the replayed step's
# per-class times); 2) kernel trace on ONE stream (MGN_CONC_WGRAD=0: every kernel on the whole chip, the
# schedule bench.py times its per-class kernels in); 3) FETCH_SIZE pass; 4) WRITE_SIZE pass; 5) SQ/GRBM
# pass (MFMA busy cycles, wave states) — separate --pmc runs, no tracing domains, on one stream too, so a
# PMC record describes the same launch bench.py's avg_launch_us times.
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
MGN_CONC_WGRAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace1 -o run -- python3 bench.py $ARGS > $OUT/trace1.log 2>&1
export MGN_CONC_WGRAD=0
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
python3 tools/pmc_traffic.py "$WL" $OUT/traffic.json $(find $OUT/fetch -name '*counter_collection.csv' | head -1) $(find $OUT/write -name '*counter_collection.csv' | head -1) $(find $OUT/sq -name '*counter_collection.csv' | head -1) $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 5 $(find $OUT/trace1 -name '*kernel_trace.csv' | head -1) "one stream (MGN_CONC_WGRAD=0)"
unset MGN_CONC_WGRAD
python3 tools/gap_summary.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 5 > $OUT/trace_summary.txt
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
echo profile-done
