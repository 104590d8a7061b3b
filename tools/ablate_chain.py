"""Diagnostic: time the chained edge-MLP kernels (forward + backward) with phases removed
(MGN_ABLATE bits: 1 input loads from HBM, 2 R8 saves, 4 MFMA, 8 row-major stores, 16 exit after weight staging). Cfg B block,
bf16 h=128. Results are wrong when a bit is set; timing only."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

ge.build()
from graphphysics import _native as nat  # noqa: E402
from graphphysics.models.layers import GraphNetBlock  # noqa: E402
from graphphysics.utils import meshes  # noqa: E402

dev = torch.device("cuda:0")
b = meshes.cylinder_batch(8, jitter=0.01)
ei = torch.from_numpy(b["edge_index"]).to(dev)
N, E, h = b["x"].shape[0], ei.shape[1], 128
torch.manual_seed(0)
blk = GraphNetBlock(h)
blk.compute_dtype = torch.bfloat16
blk = blk.to(dev)
x = torch.randn(N, h, device=dev, requires_grad=True)
e = torch.randn(E, h, device=dev, requires_grad=True)
masks = [int(v) for v in sys.argv[1:]] or [0, 1, 2, 4, 8, 2 | 8, 1 | 2 | 8, 1 | 2 | 4 | 8]
for mask in masks:
    os.environ["MGN_ABLATE"] = str(mask)
    for _ in range(3):
        x2, e2 = blk(x, ei, e)
        (x2.sum() + e2.sum()).backward()
    torch.cuda.synchronize()
    nat.profile_enable(True)
    for _ in range(10):
        x2, e2 = blk(x, ei, e)
        (x2.sum() + e2.sum()).backward()
    torch.cuda.synchronize()
    p = nat.profile_collect()
    nat.profile_enable(False)
    us = {k: 1000 * v[0] / max(v[1], 1) for k, v in p.items()}
    print(f"ablate={mask:2d}  fwd_edge {us['fwd_edge']:7.1f} us  bwd_edge {us['bwd_edge']:7.1f} us  "
          f"wgrad {us['wgrad']:6.1f}  combine {us['combine']:6.1f}  proj {us['proj']:6.1f}", flush=True)
