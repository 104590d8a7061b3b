"""Diagnostic: per-parameter gradient error of the GPU EncodeProcessDecode vs the fp64 oracle
(and the CPU fp32 oracle's own error), on the CylinderFlow mesh. Usage: diag_epd.py MP H [bf16]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
import torch  # noqa: E402

from oracle import mgn_oracle as O  # noqa: E402
from graphphysics.models.processors import EncodeProcessDecode  # noqa: E402
from graphphysics.utils import meshes  # noqa: E402
from graphphysics.utils.data import Data  # noqa: E402

DEV = torch.device("cuda:0")
mp, h = int(sys.argv[1]), int(sys.argv[2])
dt = torch.bfloat16 if len(sys.argv) > 3 else torch.float32


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


m = meshes.load_cylinder_mesh()
n = m["pos"].shape[0]
ei = torch.from_numpy(meshes.triangles_to_edge_index(m["triangles"], n))
g = torch.Generator().manual_seed(7)
x = torch.randn(n, 11, generator=g)
ea = torch.randn(ei.shape[1], 3, generator=g)
gy = torch.randn(n, 2, generator=g)
torch.manual_seed(0)
ref = O.OracleEPD(mp, 11, 3, 2, h)
rp = dict(ref.named_parameters())
yr = O.encode_process_decode(x, ei, ea, rp, mp)
(yr * gy).sum().backward()
p64 = {k: v.detach().double().requires_grad_(True) for k, v in rp.items()}
y64 = O.encode_process_decode(x.double(), ei, ea.double(), p64, mp)
(y64 * gy.double()).sum().backward()
torch.manual_seed(0)
mod = EncodeProcessDecode(mp, 11, 3, 2, h, compute_dtype=dt).to(DEV)
y = mod(Data(x=x.to(DEV), edge_index=ei.to(DEV), edge_attr=ea.to(DEV)))
(y * gy.to(DEV)).sum().backward()
print(f"y: gpu-vs-f64 {rel(y, y64):.2e} cpu32-vs-f64 {rel(yr, y64):.2e}")
for k, p in mod.named_parameters():
    print(f"{k:40s} gpu-vs-f64 {rel(p.grad, p64[k].grad):.2e}  cpu32-vs-f64 {rel(rp[k].grad, p64[k].grad):.2e}")
