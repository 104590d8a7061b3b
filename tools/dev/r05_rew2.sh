#!/bin/bash
# Round 5: REW stamps + quick A/B rows after a kernel change
set -o pipefail
bash tools/dev/r05_rst.sh 256 || exit 1
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -s \
    "tests/test_gpu_parity.py::test_recomputed_edge_weight_gradients_match_saved_inputs" > gpurun_out/rew_tests.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|rel-L2" gpurun_out/rew_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
row() {  # tag env bench-args
  env $2 timeout -k 10 300 python bench.py $3 > gpurun_out/rew_$1.log 2>&1 || { echo "$1 failed"; tail -3 gpurun_out/rew_$1.log; exit 1; }
  echo $1 $(tail -1 gpurun_out/rew_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','fwd_node','bwd_node','combine','wgrad','proj') if n in k))")
}
B="--steps 30 --warmup 5 --cpu-steps 0 --no-mse --sustain 0 --no-secondary"
row B_rew0 MGN_REW=0 "$B"
for c in 64 128 256; do row B_rew1_c$c "MGN_REW=1 MGN_REW_CHUNKS=$c" "$B"; done
E="--workload aneurysm --steps 10 --warmup 3 --cpu-steps 0 --no-mse --sustain 0 --no-secondary"
row E_rew0 MGN_REW=0 "$E"
row E_rew1_c64 "MGN_REW=1 MGN_REW_CHUNKS=64" "$E"
row E_rew1_c256 "MGN_REW=1 MGN_REW_CHUNKS=256" "$E"
