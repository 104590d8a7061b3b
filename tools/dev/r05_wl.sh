#!/bin/bash
# Round 5: LDS weight staging with the descriptor loaded in one batch (default) vs field by field in
# the layer loop (wl0): Cfg C, Cfg A, bf16 Cfg B; then the GPU tests
set -o pipefail
bash tools/dev/r05_ab.sh "--workload plate --mp 10 --hidden 64 --batch 1 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" C wl0 || exit 1
bash tools/dev/r05_ab.sh "--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" A wl0 || exit 1
bash tools/dev/r05_ab.sh "--steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3" B wl0 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wl_tests.log 2>&1; rc=$?; tail -2 gpurun_out/wl_tests.log; exit $rc
