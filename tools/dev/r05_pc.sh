#!/bin/bash
# Round 5: weight-gradient workgroups per CU for h <= 32 after the quads (MGN_WG_PER_CU32 2 default vs 1, 4): Cfg A
set -o pipefail
bash tools/dev/r05_ab.sh "--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" A pc1 pc4
