#!/bin/bash
# MGN_STAMPS variant (tools/build_variant.sh stamps "-DMGN_STAMPS"): per-phase cycle stamps of the
# chained kernels over a short bench run. bash tools/dev/stamps_run.sh <tag> [env...]
TAG=$1; shift
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_${STAMPS_VAR:-stamps}.so $L/libmgn.so
env "$@" timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --no-profile --sustain 0 $BENCH_ARGS > gpurun_out/stamps_$TAG.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
[ $rc -eq 0 ] || { tail -5 gpurun_out/stamps_$TAG.log; exit 1; }
python3 tools/stamps_summary.py gpurun_out/stamps_$TAG.log
