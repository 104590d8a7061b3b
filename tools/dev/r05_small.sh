#!/bin/bash
# Round 5: rows per workgroup of the generic kernels on the small graphs (Cfg A, Cfg C), relinked variants
set -o pipefail
bash tools/dev/r05_ab.sh "--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" A s16 s32 n16 || exit 1
bash tools/dev/r05_ab.sh "--workload plate --mp 10 --hidden 64 --batch 1 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" C s16 s32 n16
