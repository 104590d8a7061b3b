#!/bin/bash
# Round-4 breakdown: rocprofv3 trace + PMC of bf16 Cfg B, Cfg A and Cfg C (plate.json sizes), then the
# generic kernels' per-phase stamps (MGN_STAMPS variant "stm" of mgn_mlp.hip) on Cfg A and Cfg C.
#   bash tools/dev/r04_profile.sh <tag>
TAG=${1:-r04a}
bash tools/profile_round.sh $TAG && \
  bash tools/profile_round.sh ${TAG}a --mp 5 --hidden 32 --batch 1 --dtype fp32 && \
  bash tools/profile_round.sh ${TAG}p --workload plate --mp 10 --hidden 64 --batch 1 || exit 1
STAMPS_VAR=stm BENCH_ARGS="--mp 5 --hidden 32 --batch 1 --dtype fp32" bash tools/dev/stamps_run.sh ${TAG}_A > gpurun_out/stamps_${TAG}_A.txt && \
  STAMPS_VAR=stm BENCH_ARGS="--workload plate --mp 10 --hidden 64 --batch 1" bash tools/dev/stamps_run.sh ${TAG}_C > gpurun_out/stamps_${TAG}_C.txt
echo stamps=$?
# chained bf16 kernels of Cfg B: per-phase stamps and per-wave start / end spreads (variant "wt")
STAMPS_VAR=wt bash tools/dev/stamps_run.sh ${TAG}_B > gpurun_out/stamps_${TAG}_B.txt; echo stampsB=$?
bash tools/dev/wave_times.sh ${TAG}; echo wt=$?
