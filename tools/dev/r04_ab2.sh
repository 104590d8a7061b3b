#!/bin/bash
# fused node gradient: tests, then Cfg B A/B of MGN_FUSE_GRAD and the fused kernel's variants (var/*.so)
TAG=${1:-ab2}
L=graph-physics_amd/graphphysics/_lib
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "fused_node_gradient or concurrent_weight_gradients or captured_step_equals_eager or epd" \
  > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # run <label> <bench args> -- <env...>
  local lab=$1; shift; local args=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2 $args \
    > gpurun_out/ab_${TAG}_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/ab_${TAG}_$lab.log; return 1; }
  echo "$lab $(tail -1 gpurun_out/ab_${TAG}_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], (d.get('sustained') or {}).get('value'), ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad','wgrad_reduce') if n in k))")"
}
cp $L/libmgn.so /tmp/libmgn_default.so
run fuse1 "" MGN_FUSE_GRAD=1 && run fuse0 "" MGN_FUSE_GRAD=0 && run fuse1_128 "" MGN_CONC_WGRAD=128,128 && \
  run fuse1_0 "" MGN_CONC_WGRAD=0 && run fuse0_0 "" MGN_CONC_WGRAD=0 MGN_FUSE_GRAD=0 || exit 1
for v in pf1 occ3; do
  cp $L/var/libmgn_$v.so $L/libmgn.so
  run $v "" MGN_FUSE_GRAD=1; rc=$?
  cp /tmp/libmgn_default.so $L/libmgn.so
  [ $rc -eq 0 ] || exit 1
done
run fuse1b "" MGN_FUSE_GRAD=1 && run fuse0b "" MGN_FUSE_GRAD=0
