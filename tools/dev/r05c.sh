set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r05c.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_r05c.log | tail -2; grep -E "^E  |FAILED" gpurun_out/gpu_tests_r05c.log | head -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/dev/r05_ab.sh "--dtype fp32 --steps 20 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 2" f32c pn0 f32n0
