set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread "tests/test_configs_gpu.py::test_aneurysm_full_size_fp32_and_bf16_gradients" -s > gpurun_out/gpu_tests_r05d.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed|worst" gpurun_out/gpu_tests_r05d.log | tail -6
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/dev/r05_saves.sh
