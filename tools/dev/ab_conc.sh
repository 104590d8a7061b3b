#!/bin/bash
# A/B: the processor backward's weight-gradient launches on a side stream beside the next block's data
# gradients (MGN_CONC_WGRAD="data_cus,wgrad_cus") vs one stream. Headline workload only, sustained rate.
#   bash tools/dev/ab_conc.sh <tag> "192,64" "160,96" ...
TAG=$1; shift
mkdir -p gpurun_out
B="--steps 30 --warmup 5 --cpu-steps 0 --no-secondary --no-mse --no-profile --sustain 3"
for v in 0 "$@" 0; do
  MGN_CONC_WGRAD=$v timeout -k 10 200 python bench.py $B > gpurun_out/conc_${TAG}_${v/,/_}.log 2>&1 || exit 1
  python - "$v" gpurun_out/conc_${TAG}_${v/,/_}.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        print(sys.argv[1], d["value"], d["ms_per_step"], d.get("sustained"), d.get("last_loss"))
PY
done
