#!/bin/bash
# Round 5: recomputed edge weight gradients (MGN_REW) — GPU parity, then bench.py A/B rows
# (MGN_REW=0 saved R8 inputs vs 1 recomputed) at Cfg B and Cfg E.
#   bash tools/dev/r05_rew.sh [skip-tests]
set -o pipefail
mkdir -p gpurun_out
if [ "$1" != skip-tests ]; then
  timeout -k 10 400 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -s \
    "tests/test_gpu_parity.py::test_recomputed_edge_weight_gradients_match_saved_inputs" \
    "tests/test_gpu_parity.py::test_concurrent_weight_gradients_match_one_stream" \
    "tests/test_gpu_parity.py::test_deferred_weight_gradient_reduction_is_bitwise_identical" \
    > gpurun_out/rew_tests.log 2>&1
  rc=$?; echo tests=$rc; grep -E "passed|failed|rel-L2|PASSED|FAILED" gpurun_out/rew_tests.log | tail -12; grep -E "^E  " gpurun_out/rew_tests.log | head
  [ $rc -eq 0 ] || exit $rc
fi
row() {  # tag env bench-args
  env $2 timeout -k 10 300 python bench.py $3 > gpurun_out/rew_$1.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/rew_$1.log; exit 1; }
  echo $1 $(tail -1 gpurun_out/rew_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','fwd_node','bwd_node','combine','wgrad','proj') if n in k))")
}
B="--steps 30 --warmup 5 --cpu-steps 0 --no-mse --sustain 0 --no-secondary"
row B_rew0 MGN_REW=0 "$B"
for c in 64 128 256; do row B_rew1_c$c "MGN_REW=1 MGN_REW_CHUNKS=$c" "$B"; done
row B_rew1_c256_1s "MGN_REW=1 MGN_REW_CHUNKS=256 MGN_CONC_WGRAD=0" "$B"
row B_rew0_1s "MGN_REW=0 MGN_CONC_WGRAD=0" "$B"
E="--workload aneurysm --steps 10 --warmup 3 --cpu-steps 0 --no-mse --sustain 0 --no-secondary"
row E_rew0 MGN_REW=0 "$E"
row E_rew1_c256 "MGN_REW=1 MGN_REW_CHUNKS=256" "$E"
