#!/bin/bash
# Bitwise check of the current library against variant <v> (tools/dev/cmp_libs.py), then the
# headline bench A/B (tools/dev/ab_variants.sh). bash tools/dev/ab_bitwise.sh <tag> <v>
TAG=$1; V=$2
L=graph-physics_amd/graphphysics/_lib
timeout -k 10 300 python tools/dev/cmp_libs.py $L/var/libmgn_$V.so /tmp/cmp_ref.pt > gpurun_out/cmp_${TAG}_ref.log 2>&1 || { tail -5 gpurun_out/cmp_${TAG}_ref.log; exit 1; }
timeout -k 10 300 python tools/dev/cmp_libs.py $L/libmgn.so /tmp/cmp_new.pt /tmp/cmp_ref.pt > gpurun_out/cmp_${TAG}.log 2>&1 || { tail -5 gpurun_out/cmp_${TAG}.log; exit 1; }
grep "DIFF\|bitwise" gpurun_out/cmp_${TAG}.log | tail -12
bash tools/dev/ab_variants.sh $V
