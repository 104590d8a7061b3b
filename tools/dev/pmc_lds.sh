#!/bin/bash
# LDS / issue-stall counters of the training step (one --pmc pass): bash tools/pmc_lds.sh <tag>
export TMPDIR=/tmp
OUT=gpurun_out/lds_${1:-dev}
mkdir -p $OUT
ARGS="--steps 5 --warmup 3 --cpu-steps 0 --no-mse --no-profile --no-secondary --sustain 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $OUT -o run -- python3 bench.py $ARGS > $OUT/run.log 2>&1
echo pmc=$?
python3 - $OUT <<'PY'
import csv, glob, statistics, sys
sys.path.insert(0, "tools")
from pmc_traffic import kernel_class
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    c = kernel_class(r["Kernel_Name"])
    if c:
        per.setdefault((c, r["Kernel_Name"][:40]), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, v in sorted(per.items()):
    print(k[0], {n: round(statistics.median(x) / 1e6, 3) for n, x in sorted(v.items())})
PY
