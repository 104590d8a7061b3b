"""Diagnostic: bf16 gradient error of libmgn vs PyTorch CPU bf16 autocast of the reference, both
against fp64 (MP=15, h=128, cylinder)."""
import sys, os
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
import torch
import __graft_entry__ as ge
ge.build()
from oracle import mgn_oracle as O
from graphphysics.models.processors import EncodeProcessDecode
from graphphysics.utils import meshes
from graphphysics.utils.data import Data
DEV = torch.device("cuda:0")
def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()
m = meshes.load_cylinder_mesh(); n = m["pos"].shape[0]
ei = torch.from_numpy(meshes.triangles_to_edge_index(m["triangles"], n))
g = torch.Generator().manual_seed(7)
x = torch.randn(n, 11, generator=g); ea = torch.randn(ei.shape[1], 3, generator=g); gy = torch.randn(n, 2, generator=g)
torch.manual_seed(0)
ref = O.OracleEPD(15, 11, 3, 2, 128)
p64 = {k: v.detach().double().requires_grad_(True) for k, v in ref.named_parameters()}
y64 = O.encode_process_decode(x.double(), ei, ea.double(), p64, 15); (y64 * gy.double()).sum().backward()
pac = {k: v.detach().clone().requires_grad_(True) for k, v in ref.named_parameters()}
with torch.autocast("cpu", dtype=torch.bfloat16):
    yac = O.encode_process_decode(x, ei, ea, pac, 15)
(yac.float() * gy).sum().backward()
torch.manual_seed(0)
mm = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16).to(DEV)
y = mm(Data(x=x.to(DEV), edge_index=ei.to(DEV), edge_attr=ea.to(DEV))); (y * gy.to(DEV)).sum().backward()
print(f"output: autocast {rel(yac, y64):.3e}  libmgn-bf16 {rel(y, y64):.3e}")
worst = []
for k, p in mm.named_parameters():
    a, b = rel(pac[k].grad, p64[k].grad), rel(p.grad, p64[k].grad)
    worst.append((b, a, k))
for b, a, k in sorted(worst)[-8:] + sorted(worst)[:3]:
    print(f"{k:40s} autocast {a:.3e}  libmgn-bf16 {b:.3e}")
import numpy as np
print("median ratio libmgn/autocast", np.median([b / max(a, 1e-12) for b, a, k in worst]))
