#!/bin/bash
# final evidence on the final kernel sources, one GPU call: GPU suite, smoke, rocprofv3 + PMC of bf16
# Cfg B (its record copied into profiles/ so bench.py finds it by source hash), the default bench.py
# line, then rocprofv3 + PMC of fp32 Cfg B
TAG=${1:-r04d}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; tail -1 gpurun_out/gpu_tests_$TAG.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
echo smoke=ok
bash tools/profile_round.sh $TAG || exit 1
cp gpurun_out/prof_$TAG/traffic.json profiles/${TAG}_traffic.json
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1; rc=$?; echo bench=$rc
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
bash tools/profile_round.sh ${TAG}f --dtype fp32
