#!/bin/bash
# Round 6: a variant library through the GPU parity files, then a same-box A/B on one workload.
#   bash tools/dev/r06_var.sh <tag> <variant> "<test files>" "<bench args>"
TAG=$1; V=$2; TESTS=$3; ARGS=$4
L=graph-physics_amd/graphphysics/_lib
mkdir -p gpurun_out
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_$V.so $L/libmgn.so
timeout -k 10 700 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/var_tests_${TAG}.log 2>&1
rc=$?; echo tests=$rc; tail -2 gpurun_out/var_tests_${TAG}.log; grep -E "^E  " gpurun_out/var_tests_${TAG}.log | head -5
cp /tmp/libmgn_default.so $L/libmgn.so
[ $rc -eq 0 ] || exit 1
bash tools/dev/r06_ab.sh $TAG "$ARGS" $V
