#!/bin/bash
# Round 6: hidden sizes above 128 — the h = 192 / 256 parity cases on the GPU.
TAG=${1:-r06}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "192 or 256 or hidden_192" > gpurun_out/h256_$TAG.log 2>&1
rc=$?; echo tests=$rc; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/h256_$TAG.log | tail -20; grep -E "^E  " gpurun_out/h256_$TAG.log | head -20
exit $rc
