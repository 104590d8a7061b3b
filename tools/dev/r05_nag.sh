#!/bin/bash
# Round 5: chained node forward aggregation group size (MGN_NODE_AG 6 default vs 4, 3): Cfg B, Cfg E
set -o pipefail
bash tools/dev/r05_ab.sh "--steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3" B nag4 nag3 || exit 1
bash tools/dev/r05_ab.sh "--workload aneurysm --batch 1 --steps 10 --warmup 2 --cpu-steps 0 --no-mse --no-secondary --sustain 0" E nag4 || exit 1
