#!/bin/bash
# Round 5: fp32 chained edge kernels on half images, two 6-wave workgroups per CU (MGN_F32C_HALF) —
# fp32 parity, then fp32 Cfg B rows default (half) vs the 12-wave full-image variant (libmgn_half0)
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 600 --timeout-method thread \
  "tests/test_configs_gpu.py::test_aneurysm_full_size_fp32_and_bf16_gradients" tests/test_mask_pinned_gpu.py \
  tests/test_gpu_parity.py -k "fp32 or float32 or aneurysm or pinned or dtype1 or dtype2 or f32" > gpurun_out/half_tests.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" gpurun_out/half_tests.log | tail -2; grep -E "^E  " gpurun_out/half_tests.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/dev/r05_ab.sh "--dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2" half half0
