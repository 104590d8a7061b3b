#!/bin/bash
# Round 5 (reverted experiment: the MGN_F32_DENSE_BM knob was removed after this A/B, profiles/r05_ab.txt): generic fp32 dense kernels on 64-row workgroups (d64) vs 32: fp32 Cfg B, Cfg A
set -o pipefail
bash tools/dev/r05_ab.sh "--dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2" F d64 || exit 1
bash tools/dev/r05_ab.sh "--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" A d64 || exit 1
