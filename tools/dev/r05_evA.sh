#!/bin/bash
# Round 5 final evidence, part A (one GPU call): GPU suite, smoke, rocprofv3 + PMC of bf16 Cfg B and fp32
# Cfg B (records copied into profiles/ so bench.py finds them by kernel-source hash)
TAG=${1:-r05g}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; tail -1 gpurun_out/gpu_tests_$TAG.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
echo smoke=ok
bash tools/profile_round.sh $TAG || exit 1
cp gpurun_out/prof_$TAG/traffic.json profiles/${TAG}_traffic.json
bash tools/profile_round.sh ${TAG}f --dtype fp32 || exit 1
cp gpurun_out/prof_${TAG}f/traffic.json profiles/${TAG}f_traffic.json
echo evA-done
