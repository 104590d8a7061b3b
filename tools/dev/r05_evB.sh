#!/bin/bash
# Round 5 final evidence, part B (one GPU call): rocprofv3 + PMC of Cfg A, Cfg C (plate.json sizes), Cfg E
# (recomputed weight gradients on: MGN_REW=auto) and of Cfg E with MGN_REW=0 (the saves A/B, kept under
# a name bench.py does not read)
TAG=${1:-r05g}
bash tools/profile_round.sh ${TAG}a --mp 5 --hidden 32 --batch 1 --dtype fp32 && \
  bash tools/profile_round.sh ${TAG}p --workload plate --mp 10 --hidden 64 --batch 1 && \
  bash tools/profile_round.sh ${TAG}e --workload aneurysm --batch 1 || exit 1
for s in a p e; do cp gpurun_out/prof_${TAG}$s/traffic.json profiles/${TAG}${s}_traffic.json; done
MGN_REW=0 bash tools/profile_round.sh ${TAG}e0 --workload aneurysm --batch 1 || exit 1
cp gpurun_out/prof_${TAG}e0/traffic.json profiles/${TAG}e_rew0_ab.json
echo evB-done
