#!/bin/bash
# fp32 development round on the GPU box: GPU suite, fp32 gradient diagnostics against a relinked
# variant, fp32 Cfg B bench, fp32 stamps. bash tools/dev_fp32.sh <tag> <variant> <stamps-variant>
TAG=${1:-dev}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo tests=$rc; grep -E "passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -1; grep -E "^FAILED|^ERROR" gpurun_out/gpu_tests_$TAG.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/diag_chain32.sh $2 15 128 > gpurun_out/diag32_$TAG.txt 2>&1 || exit 1
head -45 gpurun_out/diag32_$TAG.txt
timeout -k 10 200 python bench.py --dtype fp32 --steps 10 --warmup 3 --cpu-steps 0 --no-mse --no-secondary --sustain 0 > gpurun_out/bench32_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench32_$TAG.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(d['value'], d['ms_per_step'], ' '.join('%s=%s' % (n, k[n]['avg_us']) for n in k))"
bash tools/stamps_var.sh $3 fp32
