#!/bin/bash
# End-of-milestone GPU evidence (run on the GPU box from the repo root): smoke, rocprofv3 trace +
# PMC passes (profiles), full bench with CPU baseline. bash tools/round_final.sh <tag>
set -e
TAG=${1:-r01}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo smoke=$?
bash tools/profile_round.sh $TAG
# the bench reports the PMC bytes of the dominant kernel when a traffic file with these sources' hash
# is under profiles/ (copied back into the repo's profiles/ after the call)
cp gpurun_out/prof_$TAG/traffic.json profiles/${TAG}_traffic.json
timeout -k 10 600 python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
echo bench=$?
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
