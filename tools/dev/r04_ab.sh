#!/bin/bash
# Round-4 A/B on one box: the fused node-gradient backward (MGN_FUSE_GRAD), CU splits of the concurrent
# backward, side-stream reductions, concurrent encoders on the small configs. Results-neutral switches.
#   bash tools/dev/r04_ab.sh <tag>
TAG=${1:-ab}
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "fused_node_gradient or concurrent_weight_gradients or captured_step_equals_eager" \
  > gpurun_out/ab_tests_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
run() {  # run <label> <bench args> -- <env...>
  local lab=$1; shift; local args=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2 $args \
    > gpurun_out/ab_${TAG}_$lab.log 2>&1 || { echo "$lab failed"; tail -3 gpurun_out/ab_${TAG}_$lab.log; return 1; }
  echo "$lab $(tail -1 gpurun_out/ab_${TAG}_$lab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], (d.get('sustained') or {}).get('value'), ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','fwd_node','bwd_edge','bwd_node','combine','wgrad','wgrad_reduce','fwd_dense','bwd_dense','wgrad_dense') if n in k))")"
}
B=""
run B_fuse1 "$B" MGN_FUSE_GRAD=1 && run B_fuse0 "$B" MGN_FUSE_GRAD=0 && \
run B_fuse1_128 "$B" MGN_FUSE_GRAD=1 MGN_CONC_WGRAD=128,128 && run B_fuse1_192 "$B" MGN_FUSE_GRAD=1 MGN_CONC_WGRAD=192,64 && \
run B_fuse1_sr "$B" MGN_FUSE_GRAD=1 MGN_SIDE_REDUCE=1 && run B_fuse0_sr "$B" MGN_FUSE_GRAD=0 MGN_SIDE_REDUCE=1 && \
run B_fuse1_b "$B" MGN_FUSE_GRAD=1 || exit 1
A="--dtype fp32 --mp 5 --hidden 32 --batch 1"
C="--workload plate --mp 10 --hidden 64 --batch 1"
run A_enc0 "$A" MGN_CONC_ENC=0 && run A_enc1 "$A" MGN_CONC_ENC=auto && \
run C_enc0 "$C" MGN_CONC_ENC=0 && run C_enc1 "$C" MGN_CONC_ENC=auto && run A_enc0b "$A" MGN_CONC_ENC=0
