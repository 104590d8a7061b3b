#!/bin/bash
# GPU suite on the shipped library, fp32 A/B against a variant, and the fp32-path GPU tests on the
# variant: bash tools/dev_ab32.sh <tag> <variant>
TAG=${1:-dev}; V=$2
L=graph-physics_amd/graphphysics/_lib
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests_$TAG.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_fp32.sh $V || exit 1
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_$V.so $L/libmgn.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "float32 or fp32 or f32 or cylinder or plate" > gpurun_out/gpu_tests_${TAG}_$V.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
echo tests_$V=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_${TAG}_$V.log | tail -1; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests_${TAG}_$V.log | head
