#!/bin/bash
# Diagnostics: relink libmgn with ONE source compiled under extra defines (A/B and ablation studies;
# never the shipped library). bash tools/build_variant.sh <name> "<defines>" [source, default mgn_chain16.hip]
set -e
L=graph-physics_amd/graphphysics/_lib
SRC=${3:-mgn_chain16.hip}
B=${SRC%.hip}
mkdir -p $L/var
EXTRA=""
[ "$SRC" = "mgn_chain16.hip" ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form"
# SRCFILE=<path>: compile that file in place of graph-physics_amd/csrc/$SRC (e.g. a `git show HEAD:...` copy)
IN=${SRCFILE:-graph-physics_amd/csrc/$SRC}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-unused-variable $EXTRA $2 -I include -I graph-physics_amd/csrc -c $IN -o $L/var/${B}_$1.o
OBJS=""
for s in mgn_mlp mgn_chain16 mgn_rew mgn_graph mgn_build mgn_prof; do
  if [ $s = $B ]; then OBJS="$OBJS $L/var/${B}_$1.o"; else OBJS="$OBJS $L/$s.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o $L/var/libmgn_$1.so
