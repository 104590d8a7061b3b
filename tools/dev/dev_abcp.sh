#!/bin/bash
# GPU suite on the shipped library, then bf16 and fp32 A/B of a relinked variant: bash tools/dev_abcp.sh <tag> <variant>
TAG=${1:-dev}; V=$2
timeout -k 10 800 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo tests=$rc; tail -1 gpurun_out/gpu_tests_$TAG.log; grep -E "^E  " gpurun_out/gpu_tests_$TAG.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab_variants.sh $V && bash tools/ab_fp32.sh $V
