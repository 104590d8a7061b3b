"""Summarise a rocprofv3 kernel trace: time per (kernel, grid) with launch counts and averages.
Usage: trace_summary.py run_kernel_trace.csv [steps]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
agg = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"][:70], r["Grid_Size_X"], r.get("Grid_Size_Y", ""))
    agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
tot = sum(sum(v) for v in agg.values())
print(f"total kernel time {tot / 1000:.2f} ms over the trace")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:30]:
    print(f"{sum(v) / tot * 100:5.1f}%  n={len(v):4d}  avg={sum(v) / len(v):8.1f} us  grid={k[1]}x{k[2]}  {k[0]}")
