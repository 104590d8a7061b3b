#!/bin/bash
# Round 5: ring job lookup unrolled over the job array (default) vs the while loop (js0): Cfg B, fp32 Cfg B, Cfg E; GPU tests
set -o pipefail
bash tools/dev/r05_ab.sh "--steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 3" B js0 || exit 1
bash tools/dev/r05_ab.sh "--dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2" F js0 || exit 1
bash tools/dev/r05_ab.sh "--workload aneurysm --batch 1 --steps 10 --warmup 2 --cpu-steps 0 --no-mse --no-secondary --sustain 0" E js0 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/js_tests.log 2>&1; rc=$?; tail -2 gpurun_out/js_tests.log; exit $rc
