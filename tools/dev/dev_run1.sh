mkdir -p gpurun_out
export MGN_TEST_RECORD_DIR=gpurun_out/rec_r04b
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_r04b.log 2>&1
echo tests=$?; tail -3 gpurun_out/gpu_tests_r04b.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-steps 0 > gpurun_out/bench_r04b.log 2>&1
echo bench=$?; tail -c 400 gpurun_out/bench_r04b.log
bash tools/dp_rehearsal.sh 4 dpb
