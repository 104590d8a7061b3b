#!/bin/bash
# Round 6: MGN_STAMPS diagnostics build of mgn_mlp.hip at fp32 Cfg B (per-phase cycles of wave 0 of WG 0).
L=graph-physics_amd/graphphysics/_lib
mkdir -p gpurun_out
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_stamps.so $L/libmgn.so
timeout -k 10 300 python bench.py --dtype fp32 --steps 3 --warmup 2 --cpu-steps 0 --no-secondary --no-mse --no-profile --sustain 0 --no-graph > gpurun_out/stamps32.log 2> gpurun_out/stamps32.err
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
python3 tools/stamps_summary.py gpurun_out/stamps32.log
exit $rc
