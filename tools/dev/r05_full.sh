#!/bin/bash
# Round 5: the whole GPU suite on the current sources (one pytest process), then smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_full.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|error" gpurun_out/gpu_tests_full.log | tail -3; grep -E "^E  |FAILED" gpurun_out/gpu_tests_full.log | head
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo smoke=$?; tail -3 gpurun_out/smoke.log
