#!/bin/bash
# GPU evidence for one milestone (run on the GPU box from the repo root): gpu tests, smoke, full bench.
#   bash tools/evidence.sh <tag>
TAG=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo smoke=$rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo bench=$rc; tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
exit $rc
