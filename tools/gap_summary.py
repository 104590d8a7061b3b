"""Per-kernel durations and inter-kernel gaps of the last `steps` replayed steps of a rocprofv3
kernel trace (one stream). Usage: gap_summary.py run_kernel_trace.csv steps"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2])
# a replayed step starts at the last `preamble_stats` launches
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("preamble_stats")]
lo = starts[-steps]
seg = rows[lo:]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(seg, seg[1:])]
print(f"steps {steps}: wall {(t1 - t0) / 1e3 / steps:.1f} us/step, kernels {busy / 1e3 / steps:.1f} us/step, "
      f"launches {len(seg) / steps:.1f}/step, mean gap {sum(gaps) / len(gaps) / 1e3:.2f} us")
agg = collections.defaultdict(list)
for r in seg:
    agg[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / steps:8.1f} us/step  n={len(v) // steps:3d}  avg={sum(v) / len(v):7.1f}  min={min(v):7.1f}  {k}")
