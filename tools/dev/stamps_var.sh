#!/bin/bash
# run a short bench on the MGN_STAMPS variant library (tools/build_variant.sh stamps "-DMGN_STAMPS")
# bash tools/stamps_var.sh [variant] [bf16|fp32]
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_${1:-stamps}.so $L/libmgn.so
timeout -k 10 200 python3 bench.py --steps 3 --warmup 2 --cpu-steps 0 --no-mse --no-profile --no-secondary --sustain 0 --dtype ${2:-bf16} > gpurun_out/stamps.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
python3 tools/stamps_summary.py gpurun_out/stamps.log
exit $rc
