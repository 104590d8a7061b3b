#!/bin/bash
# Round 5: ring chunks up to the slab capacity (Cfg E with the recomputed layers: one edge ring job)
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  "tests/test_gpu_parity.py::test_recomputed_edge_weight_gradients_match_saved_inputs" \
  "tests/test_gpu_parity.py::test_concurrent_weight_gradients_match_one_stream" \
  "tests/test_gpu_parity.py::test_deferred_weight_gradient_reduction_is_bitwise_identical" \
  "tests/test_configs_gpu.py::test_aneurysm_full_size_fp32_and_bf16_gradients" tests/test_distributed_gpu.py > gpurun_out/ringcap_tests.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" gpurun_out/ringcap_tests.log | tail -3; grep -E "^E  " gpurun_out/ringcap_tests.log | head
[ $rc -eq 0 ] || exit $rc
row() {
  env $2 timeout -k 10 300 python bench.py $3 > gpurun_out/rcap_$1.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/rcap_$1.log; exit 1; }
  echo $1 $(tail -1 gpurun_out/rcap_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','wgrad','wgrad_reduce','combine') if n in k))")
}
E="--workload aneurysm --steps 10 --warmup 3 --cpu-steps 0 --no-mse --sustain 0 --no-secondary"
row E_rew1 "MGN_REW=1" "$E"
row E_rew0 "MGN_REW=0" "$E"
B="--steps 30 --warmup 5 --cpu-steps 0 --no-mse --sustain 0 --no-secondary"
row B "MGN_REW=auto" "$B"
