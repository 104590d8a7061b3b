set -o pipefail
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread "tests/test_configs_gpu.py::test_aneurysm_full_size_fp32_and_bf16_gradients" tests/test_mask_pinned_gpu.py -s > gpurun_out/gpu_tests_r05e.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|worst|flips|PASSED|FAILED" gpurun_out/gpu_tests_r05e.log | tail -12; grep -E "^E  " gpurun_out/gpu_tests_r05e.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/dev/r05_env.sh conc "MGN_CONC_WS=3" "MGN_CONC_WGRAD=168,88" "MGN_CONC_WGRAD=152,104"
