#!/bin/bash
# Round-6 evidence in two GPU calls (each under gpurun's 20-minute limit):
#   bash tools/dev/r06_evidence.sh <tag> 1   GPU tests, smoke, Cfg B and fp32 Cfg B profiles
#   bash tools/dev/r06_evidence.sh <tag> 2   Cfg A / Cfg C / Cfg E profiles, then the default bench line
TAG=$1
mkdir -p gpurun_out
if [ "$2" = 1 ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  rc=$?; echo tests=$rc; tail -1 gpurun_out/gpu_tests_$TAG.log
  [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
  echo smoke=ok
  bash tools/profile_round.sh $TAG && bash tools/profile_round.sh ${TAG}f --dtype fp32 || exit 1
else
  bash tools/profile_round.sh ${TAG}a --mp 5 --hidden 32 --batch 1 --dtype fp32 && \
    bash tools/profile_round.sh ${TAG}p --workload plate --mp 10 --hidden 64 --batch 1 && \
    bash tools/profile_round.sh ${TAG}e --workload aneurysm --batch 1 || exit 1
  for s in "" f a p e; do [ -f gpurun_out/prof_${TAG}$s/traffic.json ] && cp gpurun_out/prof_${TAG}$s/traffic.json profiles/${TAG}${s}_traffic.json; done
  timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo bench=$rc; tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json; exit $rc
fi
