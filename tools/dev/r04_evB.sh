#!/bin/bash
# final evidence, part B: rocprofv3 + PMC of Cfg A, Cfg C (plate.json sizes), Cfg E; the bench line
# (reads profiles/<tag>*_traffic.json by source hash); the N>1 rehearsal (4 gloo ranks on one GPU) and
# the 1-rank RCCL data-parallel step
TAG=${1:-r04c}
bash tools/profile_round.sh ${TAG}a --mp 5 --hidden 32 --batch 1 --dtype fp32 && \
  bash tools/profile_round.sh ${TAG}p --workload plate --mp 10 --hidden 64 --batch 1 && \
  bash tools/profile_round.sh ${TAG}e --workload aneurysm --batch 1 || exit 1
for s in a p e; do cp gpurun_out/prof_${TAG}$s/traffic.json profiles/${TAG}${s}_traffic.json; done
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1; rc=$?; echo bench=$rc
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
bash tools/dp_rehearsal.sh 4 dp_$TAG
