set -o pipefail
timeout -k 10 700 python -u -m pytest -x -v -p no:cacheprovider --timeout 600 --timeout-method thread "tests/test_configs_gpu.py::test_aneurysm_full_size_fp32_and_bf16_gradients" tests/test_mask_pinned_gpu.py tests/test_rollout_gpu.py -s > gpurun_out/gpu_tests_r05f.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|worst|flips|PASSED|FAILED" gpurun_out/gpu_tests_r05f.log | tail -14; grep -E "^E  " gpurun_out/gpu_tests_r05f.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/dev/r05_saves.sh
