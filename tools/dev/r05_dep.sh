#!/bin/bash
# Round 5: device-side hand-over in the concurrent backward (MGN_BLOCK_DEP) — parity / schedule tests,
# then same-box rows: events vs device hand-over, workspace rotation 2 vs 3
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_block_dep_handover_equals_event_ordering" \
  "tests/test_gpu_parity.py::test_concurrent_weight_gradients_match_one_stream" \
  "tests/test_gpu_parity.py::test_captured_step_equals_eager_step" tests/test_step_gpu.py tests/test_distributed_gpu.py \
  > gpurun_out/dep_tests.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" gpurun_out/dep_tests.log | tail -2; grep -E "^E  |FAILED|timed out" gpurun_out/dep_tests.log | head
[ $rc -eq 0 ] || exit $rc
bash tools/dev/r05_env.sh dep "MGN_BLOCK_DEP=0" "MGN_BLOCK_DEP=1 MGN_CONC_WS=3" "MGN_BLOCK_DEP=0"
