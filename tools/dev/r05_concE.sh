#!/bin/bash
# Round 5: Cfg E on the concurrent backward at 128 + 128 CUs ("auto"), vs one stream; then the GPU tests
set -o pipefail
bash tools/dev/r05_envE.sh auto "MGN_CONC_WGRAD=0" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/concE_tests.log 2>&1; rc=$?; tail -2 gpurun_out/concE_tests.log; exit $rc
