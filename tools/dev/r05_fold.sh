#!/bin/bash
# Round 5: fp32 node forward with the next block's projections (fold) — fp32 parity tests + fp32 Cfg B rows
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -s \
  "tests/test_configs_gpu.py::test_aneurysm_full_size_fp32_and_bf16_gradients" tests/test_mask_pinned_gpu.py \
  "tests/test_gpu_parity.py" -k "fp32 or float32 or aneurysm or pinned or dtype1 or dtype2 or f32" > gpurun_out/fold_tests.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|worst pinned" gpurun_out/fold_tests.log | tail -6; grep -E "^E  " gpurun_out/fold_tests.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 0 > gpurun_out/fold_f32_$i.log 2>&1 || exit 3
tail -1 gpurun_out/fold_f32_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('fold', d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in ('fwd_node','proj','bwd_node') if n in k))"
done
