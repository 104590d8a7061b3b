"""Median per-phase s_memtime deltas of MGN_STAMPS builds (one line per kernel launch, wave 0 of
workgroup 0): python3 tools/stamps_summary.py gpurun_out/stamps.log"""
import sys
from collections import defaultdict

rows = defaultdict(list)
for line in open(sys.argv[1], errors="replace"):
    p = line.split()
    if len(p) == 13 and p[0] in ("fwd16", "bwd16", "nfwd16", "nbwd16", "f32f", "f32b", "gfe", "gfn", "gfd", "gbe", "gbn", "gwg", "f32nf", "f32nb"):
        rows[p[0]].append([int(v) for v in p[1:]])
stage = sorted(int(l.split()[1]) for l in open(sys.argv[1], errors="replace") if l.startswith("nfwd16_stage "))
if stage:
    print(f"nfwd16 staging (stager wave 4 of WG 0): median {stage[len(stage) // 2]} cycles over {len(stage)} launches")
for name, rs in rows.items():
    med = [sorted(c)[len(c) // 2] for c in zip(*rs)]
    print(f"{name:7s} n={len(rs):3d} total={sum(med):6d}  " + " ".join(f"{v:6d}" for v in med))
