#!/bin/bash
# Round 5: per-kernel L1 accesses per vector load / TA busy (address-bound kernels), one workload per arg
set -o pipefail
O=gpurun_out/acc; mkdir -p $O
run() {
  T=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc TA_BUSY_avr SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $O/${T}_p2 -o run -- python3 bench.py "$@" > $O/${T}_p2.log 2>&1 && \
  timeout -s KILL 150 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/${T}_p3 -o run -- python3 bench.py "$@" > $O/${T}_p3.log 2>&1
}
C="--steps 3 --warmup 1 --cpu-steps 0 --no-mse --no-secondary --sustain 0 --no-profile"
run B $C && run C --workload plate --mp 10 --hidden 64 --batch 1 $C && run F --dtype fp32 $C && run A --mp 5 --hidden 32 --batch 1 --dtype fp32 $C
rc=$?; echo rc=$rc; exit $rc
