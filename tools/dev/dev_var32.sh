#!/bin/bash
# fp32 A/B of a relinked variant plus the fp32-path GPU tests on it: bash tools/dev_var32.sh <variant>
V=$1
L=graph-physics_amd/graphphysics/_lib
bash tools/ab_fp32.sh $V || exit 1
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_$V.so $L/libmgn.so
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "float32 or fp32 or f32 or cylinder or plate" > gpurun_out/gpu_tests_var_$V.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
echo tests_$V=$rc; tail -1 gpurun_out/gpu_tests_var_$V.log; grep -E "^E  " gpurun_out/gpu_tests_var_$V.log | head -5
