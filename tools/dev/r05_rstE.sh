#!/bin/bash
# Round 5: recompute-kernel per-phase stamps at Cfg E (libmgn_rst variant: -DMGN_STAMPS on mgn_rew.hip), one stream
set -o pipefail
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_rst.so $L/libmgn.so
MGN_REW=1 MGN_CONC_WGRAD=0 timeout -k 10 300 python bench.py --workload aneurysm --steps 2 --warmup 1 --cpu-steps 0 --no-mse --sustain 0 --no-secondary --no-profile > gpurun_out/rstE.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
echo rc=$rc; grep "^rew w" gpurun_out/rstE.log | tail -24
