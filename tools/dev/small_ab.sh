#!/bin/bash
# Small-graph rows (Cfg A, Cfg C at plate.json's sizes) for the current library and, with a variant
# name, for graph-physics_amd/graphphysics/_lib/var/libmgn_<name>.so; bitwise check vs that variant.
#   bash tools/dev/small_ab.sh <tag> [variant]
TAG=$1; V=$2
L=graph-physics_amd/graphphysics/_lib
mkdir -p gpurun_out
run() {
  for w in "A:--dtype fp32 --mp 5 --hidden 32 --batch 1" "C:--workload plate --mp 10 --hidden 64 --batch 1"; do
    t=${w%%:*}; args=${w#*:}
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-steps 0 --no-mse --no-secondary --sustain 2 $args > gpurun_out/small_${TAG}_$1_$t.log 2>&1 || return 1
    echo "$1 $t $(tail -1 gpurun_out/small_${TAG}_$1_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], (d.get('sustained') or {}).get('value'), ' '.join('%s=%s' % (n, v['avg_us']) for n, v in k.items()))")"
  done
}
if [ -n "$V" ]; then
  timeout -k 10 300 python tools/dev/cmp_libs.py $L/var/libmgn_$V.so /tmp/cmp_ref.pt > gpurun_out/cmp_${TAG}_ref.log 2>&1 || { tail -5 gpurun_out/cmp_${TAG}_ref.log; exit 1; }
  timeout -k 10 300 python tools/dev/cmp_libs.py $L/libmgn.so /tmp/cmp_new.pt /tmp/cmp_ref.pt > gpurun_out/cmp_${TAG}.log 2>&1 || { tail -5 gpurun_out/cmp_${TAG}.log; exit 1; }
  tail -12 gpurun_out/cmp_${TAG}.log
  cp $L/libmgn.so /tmp/libmgn_cur.so
  cp $L/var/libmgn_$V.so $L/libmgn.so
  run $V; rc=$?
  cp /tmp/libmgn_cur.so $L/libmgn.so
  [ $rc -eq 0 ] || exit 1
fi
run cur
