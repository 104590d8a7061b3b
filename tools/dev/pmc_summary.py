"""Average PMC counters per (kernel, grid) from a rocprofv3 counter_collection.csv."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    key = (r["Kernel_Name"][:60], r.get("Grid_Size", r.get("Grid_Size_X", "")))
    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):14.0f}  (n={len(v)})")
