#!/bin/bash
# The whole -m gpu suite (one process) + smoke(): bash tools/dev/gpu_suite.sh <tag>
TAG=$1
mkdir -p gpurun_out
export MGN_TEST_RECORD_DIR=gpurun_out/rec_$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; rc=$?
tail -2 gpurun_out/smoke_$TAG.log
exit $rc
