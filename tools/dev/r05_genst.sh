#!/bin/bash
# Round 5: per-phase stamps of the generic kernels (libmgn_st: -DMGN_STAMPS on mgn_mlp.hip), Cfg C and Cfg A, 2 steps
set -o pipefail
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
cp $L/var/libmgn_st.so $L/libmgn.so
timeout -k 10 300 python bench.py --workload plate --mp 10 --hidden 64 --batch 1 --steps 2 --warmup 1 --cpu-steps 0 --no-mse --no-secondary --sustain 0 --no-profile > gpurun_out/genst_C.log 2>&1 && \
timeout -k 10 300 python bench.py --mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 2 --warmup 1 --cpu-steps 0 --no-mse --no-secondary --sustain 0 --no-profile > gpurun_out/genst_A.log 2>&1
rc=$?
cp /tmp/libmgn_default.so $L/libmgn.so
echo rc=$rc; grep -c "^g" gpurun_out/genst_C.log gpurun_out/genst_A.log
