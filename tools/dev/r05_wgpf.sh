#!/bin/bash
# Round 5: fp32 generic weight gradients on 16-byte row quads (default) vs the committed kernel (old):
# Cfg A, Cfg C, fp32 Cfg B, then the GPU tests
set -o pipefail
bash tools/dev/r05_ab.sh "--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" A old || exit 1
bash tools/dev/r05_ab.sh "--dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2" F old || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wgpf_tests.log 2>&1; rc=$?; tail -2 gpurun_out/wgpf_tests.log; exit $rc
