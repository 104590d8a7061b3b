#!/bin/bash
# A/B of every bench row (headline + secondary) for MGN_CONC_WGRAD settings.
#   bash tools/dev/ab_conc_all.sh <tag> 0 auto ...
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  MGN_CONC_WGRAD=$v timeout -k 10 400 python bench.py --steps 30 --warmup 5 --cpu-steps 0 --no-mse --no-profile --sustain 2 > gpurun_out/concall_${TAG}_${v/,/_}.log 2>&1 || exit 1
  python - "$v" gpurun_out/concall_${TAG}_${v/,/_}.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{"):
        d = json.loads(l)
        row = {"B": (d["value"], (d.get("sustained") or {}).get("value"))}
        for k, v in d.get("secondary", {}).items():
            row[k] = v.get("value")
        print(sys.argv[1], row)
PY
done
