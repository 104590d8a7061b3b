#!/bin/bash
# Round 5: bf16 generic kernels on 32-row edge/dense and 16-row node workgroups — the GPU suite, then
# same-box rows against the previous tiles (libmgn_old: 64 / 32) on Cfg C, Cfg A, Cfg B
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/bm_tests.log 2>&1
rc=$?; echo tests=$rc; tail -1 gpurun_out/bm_tests.log; grep -E "^E  |FAILED" gpurun_out/bm_tests.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/dev/r05_ab.sh "--workload plate --mp 10 --hidden 64 --batch 1 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" Cbm old || exit 1
bash tools/dev/r05_ab.sh "--steps 30 --warmup 5 --cpu-steps 0 --no-mse --no-secondary --sustain 2" Bbm old
