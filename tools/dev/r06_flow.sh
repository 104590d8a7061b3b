#!/bin/bash
# Round 6: flag-synchronized fp32 edge forward (MGN_F32C_FLOW variant build) — fp32 parity tests on the
# variant, then fp32 Cfg B A/B (default vs flow) on one box.   bash tools/dev/r06_flow.sh <tag> [variants...]
TAG=$1; shift
L=graph-physics_amd/graphphysics/_lib
cp $L/libmgn.so /tmp/libmgn_default.so
for v in "$@"; do
  cp $L/var/libmgn_$v.so $L/libmgn.so
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mask_pinned_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "float32 or fp32 or f32 or mask" > gpurun_out/flow_tests_${TAG}_$v.log 2>&1
  rc=$?; echo tests_$v=$rc; tail -2 gpurun_out/flow_tests_${TAG}_$v.log
  [ $rc -eq 0 ] || { cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
done
for v in default "$@" default "$@"; do
  if [ $v = default ]; then cp /tmp/libmgn_default.so $L/libmgn.so; else cp $L/var/libmgn_$v.so $L/libmgn.so; fi
  timeout -k 10 300 python bench.py --dtype fp32 --steps 10 --warmup 3 --cpu-steps 0 --no-secondary --no-mse --sustain 0 > gpurun_out/flow_${TAG}_$v.json 2> gpurun_out/flow_${TAG}_$v.err || { cp /tmp/libmgn_default.so $L/libmgn.so; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/flow_${TAG}_$v.json'))
k=d['kernels']; print('$v', d['value'], d['ms_per_step'], ' '.join('%s=%.1f' % (c, k[c]['avg_us']) for c in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad') if c in k))"
done
cp /tmp/libmgn_default.so $L/libmgn.so
