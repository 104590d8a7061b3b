#!/bin/bash
# Round 5: DP/step GPU tests, single-process vs 1-rank RCCL data-parallel step (x2, same box), 4-rank gloo rehearsal.
TAG=${1:-r05dp2}
O=gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_step_gpu.py tests/test_distributed_gpu.py "tests/test_gpu_parity.py::test_eager_between_replays_keeps_graph_gradients" \
  > $O/tests_$TAG.log 2>&1
rc=$?; echo tests=$rc; grep -E "passed|failed" $O/tests_$TAG.log | tail -2; grep -E "^E  |Warning" $O/tests_$TAG.log | head -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-profile --no-mse --no-secondary --sustain 3 > $O/bench1_${TAG}_$i.log 2>&1 || exit 3
timeout -k 10 240 python bench.py --dp --steps 20 --warmup 3 --cpu-steps 0 --no-profile --no-mse --no-secondary --sustain 3 > $O/benchdp_${TAG}_$i.log 2>&1 || exit 4
for f in $O/bench1_${TAG}_$i.log $O/benchdp_${TAG}_$i.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['sustained']['value'], d['execution'][:60])"; done
done
bash tools/dp_rehearsal.sh 4 dp_$TAG
