#!/bin/bash
# Per-step kernel inventory of the replayed training step: kernel traces of two bench runs that differ
# only in the number of timed steps; (counts, time) of run B minus run A, divided by the step difference.
export TMPDIR=/tmp
rm -rf gpurun_out/ts; mkdir -p gpurun_out/ts
for s in 5 25; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ts/s$s -o run -- python3 bench.py --steps $s --warmup 3 --cpu-steps 0 --no-mse --no-profile > gpurun_out/ts/log$s 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
def load(s):
    f = glob.glob(f"gpurun_out/ts/s{s}/**/*kernel_trace.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:90], r["Grid_Size_X"])
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    return agg
a, b = load(5), load(25)
rows = []
for k in set(a) | set(b):
    n = (b[k][0] - a[k][0]) / 20
    t = (b[k][1] - a[k][1]) / 20
    if n > 0.01:
        rows.append((t, n, k))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
with open("gpurun_out/ts/per_step.txt", "w") as f:
    f.write(f"per-step kernel time {tot:.1f} us in {sum(r[1] for r in rows):.1f} launches\n")
    for t, n, k in rows:
        f.write(f"{t:8.1f} us {n:6.2f}/step avg {t / n:6.1f}  grid={k[1]}  {k[0]}\n")
print(open("gpurun_out/ts/per_step.txt").read())
PY
