#!/bin/bash
# bash tools/dev/wave_times.sh <tag> [env...]: tools/dev/wave_times.py on the MGN_STAMPS variant "wt"
TAG=$1; shift
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_wt.so $L/libmgn.so
env "$@" timeout -k 10 200 python tools/dev/wave_times.py > gpurun_out/wt_$TAG.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
grep -v "^fwd16\|^bwd16\|^nfwd16\|^nbwd16\|^gf\|^gb\|^gw" gpurun_out/wt_$TAG.log | tail -8
exit $rc
