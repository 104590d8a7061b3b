#!/bin/bash
# Round 5: generic node forward aggregation in clamped groups of 8 in-edges (default) vs groups of 4
# (ag4) vs the committed form (old: groups of 4 + one edge at a time), Cfg C and Cfg A; then GPU tests
set -o pipefail
bash tools/dev/r05_ab.sh "--workload plate --mp 10 --hidden 64 --batch 1 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" C old ag4 || exit 1
bash tools/dev/r05_ab.sh "--mp 5 --hidden 32 --batch 1 --dtype fp32 --steps 200 --warmup 20 --cpu-steps 0 --no-mse --no-secondary --sustain 2" A old || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ag_tests.log 2>&1; rc=$?; tail -2 gpurun_out/ag_tests.log; exit $rc
