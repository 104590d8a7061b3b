#!/bin/bash
# Whole round-end evidence in one GPU call: tools/evidence_profiles.sh <tag> (tests, smoke, 4 profiled
# workloads), the PMC records copied into profiles/ for bench.py, then the default bench line.
TAG=${1:-r04}
bash tools/evidence_profiles.sh $TAG || exit 1
for s in "" f a p e; do cp gpurun_out/prof_${TAG}$s/traffic.json profiles/${TAG}${s}_traffic.json; done
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo bench=$rc; tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json; exit $rc
