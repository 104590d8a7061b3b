#!/bin/bash
# Round 5: recompute kernel change — parity, Cfg E stamps, Cfg E rows
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_recomputed_edge_weight_gradients_match_saved_inputs" > gpurun_out/rew3_tests.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" gpurun_out/rew3_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
bash tools/dev/r05_rstE.sh | tail -12 || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --workload aneurysm --steps 10 --warmup 3 --cpu-steps 0 --no-mse --sustain 0 --no-secondary > gpurun_out/rew3_E_$i.log 2>&1 || exit 3
tail -1 gpurun_out/rew3_E_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('E', d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_edge','bwd_edge','wgrad','wgrad_reduce') if n in k))"
done
