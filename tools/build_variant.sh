#!/bin/bash
# Diagnostics: relink libmgn with mgn_chain16.hip compiled under extra defines (A/B and ablation
# studies; never the shipped library). bash tools/build_variant.sh <name> "<defines>"
set -e
L=graph-physics_amd/graphphysics/_lib
mkdir -p $L/var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable -mllvm -amdgpu-mfma-vgpr-form $2 -I include -c graph-physics_amd/csrc/mgn_chain16.hip -o $L/var/chain16_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $L/mgn_mlp.o $L/var/chain16_$1.o $L/mgn_graph.o $L/mgn_build.o $L/mgn_prof.o -o $L/var/libmgn_$1.so
