"""Diagnostic: GPU fp32/bf16 block vs CPU fp32 oracle vs fp64 oracle (truth)."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
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
h = 128
torch.manual_seed(0)
blk = GraphNetBlock(h)
g = torch.Generator().manual_seed(1234)
x = torch.randn(n, h, generator=g); e = torch.randn(ei.shape[1], h, generator=g)
gx = torch.randn(n, h, generator=g); ge_ = torch.randn(ei.shape[1], h, generator=g)
res = {}
for tag, dt in (("cpu32", torch.float32), ("f64", torch.float64)):
    rp = {k: v.detach().clone().to(dt).detach().requires_grad_(True) for k, v in blk.named_parameters()}
    xr, er = x.clone().to(dt).detach().requires_grad_(True), e.clone().to(dt).detach().requires_grad_(True)
    x2r, e2r = O.graph_net_block(xr, ei, er, rp)
    ((x2r * gx.to(dt)).sum() + (e2r * ge_.to(dt)).sum()).backward()
    res[tag] = dict(x=x2r, e=e2r, dx=xr.grad, de=er.grad, **{k: v.grad for k, v in rp.items()})
for cdt in (torch.float32, torch.bfloat16):
    b = GraphNetBlock(h); b.load_state_dict(blk.state_dict()); b.compute_dtype = cdt; b = b.to(DEV)
    xd, ed = x.to(DEV).detach().requires_grad_(True), e.to(DEV).detach().requires_grad_(True)
    x2, e2 = b(xd, ei.to(DEV), ed)
    ((x2 * gx.to(DEV)).sum() + (e2 * ge_.to(DEV)).sum()).backward()
    res[str(cdt)] = dict(x=x2, e=e2, dx=xd.grad, de=ed.grad, **{k: v.grad for k, v in b.named_parameters()})
for key in res["f64"]:
    print(f"{key:28s} cpu32-vs-f64 {rel(res['cpu32'][key], res['f64'][key]):.2e}  gpu32-vs-f64 {rel(res[str(torch.float32)][key], res['f64'][key]):.2e}  gpubf16-vs-f64 {rel(res[str(torch.bfloat16)][key], res['f64'][key]):.2e}  gpu32-vs-cpu32 {rel(res[str(torch.float32)][key], res['cpu32'][key]):.2e}")
