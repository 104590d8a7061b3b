#!/bin/bash
# Round 5: Cfg A counters for the generic weight-gradient launch (TLB, L1->L2 latency, TA), separate passes
set -o pipefail
A="--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 5 --warmup 2 --cpu-steps 0 --no-mse --no-secondary --sustain 0 --no-profile"
O=gpurun_out/wgpmc; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --output-format csv -d $O/p1 -o run -- python3 bench.py $A > $O/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 bench.py $A > $O/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum --output-format csv -d $O/p3 -o run -- python3 bench.py $A > $O/p3.log 2>&1
rc=$?; echo rc=$rc; tail -2 $O/p1.log $O/p2.log $O/p3.log; exit $rc
