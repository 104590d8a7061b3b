"""Diagnostic: per-component backward error of one GraphNetBlock vs the oracle."""
import sys, os
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-physics_amd")]
import torch
import __graft_entry__ as ge
ge.build()
from oracle import mgn_oracle as O
from graphphysics.models.layers import GraphNetBlock
from graphphysics.utils import meshes
DEV = torch.device("cuda:0")

def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()

m = meshes.load_cylinder_mesh(); n = m["pos"].shape[0]
ei = torch.from_numpy(meshes.triangles_to_edge_index(m["triangles"], n))
for h in (16, 32, 64, 128):
    for mode in ("x", "e"):
        torch.manual_seed(0)
        blk = GraphNetBlock(h)
        rp = {k: v.detach().clone().requires_grad_(True) for k, v in blk.named_parameters()}
        g = torch.Generator().manual_seed(1234)
        x = torch.randn(n, h, generator=g); e = torch.randn(ei.shape[1], h, generator=g)
        gx = torch.randn(n, h, generator=g) if mode == "x" else torch.zeros(n, h)
        ge_ = torch.randn(ei.shape[1], h, generator=g) if mode == "e" else torch.zeros(ei.shape[1], h)
        xr, er = x.clone().requires_grad_(True), e.clone().requires_grad_(True)
        x2r, e2r = O.graph_net_block(xr, ei, er, rp)
        ((x2r * gx).sum() + (e2r * ge_).sum()).backward()
        blk.compute_dtype = torch.float32; blk = blk.to(DEV)
        xd, ed = x.to(DEV).requires_grad_(True), e.to(DEV).requires_grad_(True)
        x2, e2 = blk(xd, ei.to(DEV), ed)
        ((x2 * gx.to(DEV)).sum() + (e2 * ge_.to(DEV)).sum()).backward()
        d = (xd.grad.cpu() - xr.grad).abs()
        rowerr = d.max(1).values
        print(f"h={h} loss-on-{mode}: fwd x {rel(x2, x2r):.2e} e {rel(e2, e2r):.2e} | dx {rel(xd.grad, xr.grad):.2e} de {rel(ed.grad, er.grad):.2e}",
              " worst rows", rowerr.topk(3).indices.tolist(), [f"{v:.2e}" for v in rowerr.topk(3).values.tolist()],
              "xgrad scale", xr.grad.abs().max().item())
        print("   params:", " ".join(f"{k.split('.')[0][0]}{k.split('.')[1]}{k.split('.')[2][0]}={rel(p.grad, rp[k].grad):.1e}" for k, p in blk.named_parameters()))
