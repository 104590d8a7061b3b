"""Diagnostic: one GraphNetBlock (bf16 h=128) forward+backward on the Cfg B batch; saves outputs
and gradients to gpurun_out/chain_<MGN_CHAIN>.pt; with two files present, compares them."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

ge.build()
from graphphysics.models.layers import GraphNetBlock  # noqa: E402
from graphphysics.utils import meshes  # noqa: E402

dev = torch.device("cuda:0")
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 8
b = meshes.cylinder_batch(nb, jitter=0.01)
ei = torch.from_numpy(b["edge_index"]).to(dev)
N, E, h = b["x"].shape[0], ei.shape[1], 128
torch.manual_seed(0)
blk = GraphNetBlock(h)
blk.compute_dtype = torch.bfloat16
blk = blk.to(dev)
g = torch.Generator().manual_seed(1)
x = torch.randn(N, h, generator=g).to(dev).requires_grad_(True)
e = torch.randn(E, h, generator=g).to(dev).requires_grad_(True)
gx, ge_ = torch.randn(N, h, generator=g).to(dev), torch.randn(E, h, generator=g).to(dev)
x2, e2 = blk(x, ei, e)
((x2 * gx).sum() + (e2 * ge_).sum()).backward()
res = {"x2": x2.detach().cpu(), "e2": e2.detach().cpu(), "dx": x.grad.cpu(), "de": e.grad.cpu(),
       **{k: p.grad.cpu() for k, p in blk.named_parameters()}}
tag = os.environ.get("MGN_CHAIN", "32")
os.makedirs("gpurun_out", exist_ok=True)
torch.save(res, f"gpurun_out/chain_{tag}_{nb}.pt")
other = f"gpurun_out/chain_{'32' if tag == '16' else '16'}_{nb}.pt"
if os.path.exists(other):
    o = torch.load(other, weights_only=True)
    for k, v in res.items():
        d = (v.double() - o[k].double()).norm() / (o[k].double().norm() + 1e-30)
        fin = bool(torch.isfinite(v).all())
        print(f"{k:28s} rel {d.item():.3e} finite {fin}")
