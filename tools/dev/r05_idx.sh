#!/bin/bash
# Round 5: node_grad's source-direction edge ids prefetched a group ahead (default) vs not (idx0): Cfg E, Cfg B
set -o pipefail
bash tools/dev/r05_ab.sh "--workload aneurysm --batch 1 --steps 10 --warmup 2 --cpu-steps 0 --no-mse --no-secondary --sustain 0" E idx0 || exit 1
bash tools/dev/r05_ab.sh "--steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3" B idx0 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/idx_tests.log 2>&1; rc=$?; tail -2 gpurun_out/idx_tests.log; exit $rc
