#!/bin/bash
# Round 5 final evidence, part C (one GPU call): the default bench.py line (reads the profiles/ records),
# single-process vs 1-rank RCCL data-parallel step on the same box, the 4-rank gloo rehearsal
TAG=${1:-r05g}
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1; rc=$?; echo bench=$rc
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 240 python bench.py --steps 20 --warmup 3 --cpu-steps 0 --no-profile --no-mse --no-secondary --sustain 3 > gpurun_out/bench1_${TAG}_$i.log 2>&1 || exit 3
timeout -k 10 240 python bench.py --dp --steps 20 --warmup 3 --cpu-steps 0 --no-profile --no-mse --no-secondary --sustain 3 > gpurun_out/benchdp_${TAG}_$i.log 2>&1 || exit 4
done
bash tools/dp_rehearsal.sh 4 dp_$TAG
echo evC-done
