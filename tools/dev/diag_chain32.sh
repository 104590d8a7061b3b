#!/bin/bash
# fp32 EncodeProcessDecode per-parameter gradient errors vs fp64 (tools/diag_epd.py) with the shipped
# library and with a relinked variant (tools/build_variant.sh): bash tools/diag_chain32.sh <variant> MP H
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
timeout -k 10 300 python3 tools/diag_epd.py $2 $3 > gpurun_out/diag_default.log 2>&1
rc=$?
cp $L/var/libmgn_$1.so $L/libmgn.so
timeout -k 10 300 python3 tools/diag_epd.py $2 $3 > gpurun_out/diag_$1.log 2>&1
rc2=$?
cp /tmp/libmgn_default.so $L/libmgn.so
echo rc=$rc rc2=$rc2
paste <(awk '{print $1, $3}' gpurun_out/diag_default.log) <(awk '{print $3, $5}' gpurun_out/diag_$1.log) | sort -k2 -g -r | head -40
