#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: N ranks (default 4) sharing cuda:0, gloo exchanges (RCCL
# needs one GPU per rank). Checks that the data-parallel step runs end to end — every rank agrees on
# world size / parameters / gradient-bucket coverage (bench.py raises otherwise) — and prints one JSON line.
#   bash tools/dp_rehearsal.sh [N] [tag]
N=${1:-4}
TAG=${2:-dp}
MGN_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $N --steps 10 --warmup 3 --no-profile --sustain 1 > gpurun_out/${TAG}$N.log 2>gpurun_out/${TAG}$N.err
echo dp$N=$?
tail -1 gpurun_out/${TAG}$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['optimizer_steps_per_s'], d['ms_per_step'], d['n_gpus'], d.get('data_parallel'), d.get('one_step_mse'))"
# 1 rank through the same data-parallel step (RCCL group of one: the overlapped all-reduce in the graph)
timeout -k 10 300 python bench.py --dp --steps 20 --warmup 3 --cpu-steps 0 --no-profile --no-mse > gpurun_out/${TAG}1.log 2>&1
echo dp1=$?
tail -1 gpurun_out/${TAG}1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['execution'])"
