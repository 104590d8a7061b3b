#!/bin/bash
# Round 5: training-mode vs inference-mode block forward (saves vs none) at Cfg B and Cfg E, HIP-event
# per-class times and PMC bytes per kernel instance (FETCH_SIZE / WRITE_SIZE passes of their own).
export TMPDIR=/tmp
O=gpurun_out/saves
mkdir -p $O
for w in cylinder aneurysm; do
  timeout -k 10 200 python tools/dev/r05_saves.py $w 20 > $O/times_$w.json 2> $O/times_$w.err || exit 3
  cat $O/times_$w.json
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$w -o run -- python3 tools/dev/r05_saves.py $w 5 > $O/fetch_$w.log 2>&1 || exit 4
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$w -o run -- python3 tools/dev/r05_saves.py $w 5 > $O/write_$w.log 2>&1 || exit 5
  python3 - $w <<'PY'
import csv, glob, statistics, sys
w = sys.argv[1]
out = {}
for kind, cnt in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
    f = glob.glob("gpurun_out/saves/%s_%s/**/*counter_collection.csv" % (kind, w), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "chain16_fwd_kernel" in n and r["Counter_Name"] == cnt:
            key = "train" if "<true" in n else "infer"
            per.setdefault(key, []).append(float(r["Counter_Value"]) * 1024 * (2.0 if kind == "fetch" else 1.0))
    for k, v in per.items():
        out.setdefault(k, {})[kind + "_MB"] = round(statistics.median(v) / 1e6, 1)
print(w, out)
PY
done
