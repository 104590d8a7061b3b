#!/bin/bash
# Round evidence, part 1 (GPU box, repo root): GPU test suite, smoke, rocprofv3 trace + PMC passes for
# the headline workload and the secondary rows (fp32 Cfg B, Cfg A, Cfg C at plate.json's sizes, Cfg E).
# bash tools/evidence_profiles.sh <tag>   -> gpurun_out/{gpu_tests,smoke}_<tag>.log, prof_<tag>{,f,a,p,e}/
TAG=${1:-r03b}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo tests=$rc; tail -1 gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
echo smoke=ok
bash tools/profile_round.sh $TAG && bash tools/profile_round.sh ${TAG}f --dtype fp32 && \
  bash tools/profile_round.sh ${TAG}a --mp 5 --hidden 32 --batch 1 --dtype fp32 && \
  bash tools/profile_round.sh ${TAG}p --workload plate --mp 10 --hidden 64 --batch 1 && \
  bash tools/profile_round.sh ${TAG}e --workload aneurysm --batch 1
