#!/bin/bash
# small-graph A/B: current library vs var/libmgn_old.so (bitwise comparison + Cfg A / Cfg C rows), then
# the GPU parity tests of the generic kernels
TAG=${1:-ab3}
bash tools/dev/small_ab.sh $TAG old || exit 1
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests_$TAG.log; exit $rc
