"""Diagnostic: fp32 EncodeProcessDecode (MP=5, h=32, cylinder mesh, seed 7) per-parameter gradient
errors vs fp64, plus where the node encoder's layer-0 weight gradient differs most."""
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
p64 = {k: v.detach().double().requires_grad_(True) for k, v in rp.items()}
y64 = O.encode_process_decode(x.double(), ei, ea.double(), p64, mp)
(y64 * gy.double()).sum().backward()
torch.manual_seed(0)
mod = EncodeProcessDecode(mp, 11, 3, 2, h, compute_dtype=torch.float32).to(DEV)
for it in range(2):
    mod.zero_grad(set_to_none=True)
    y = mod(Data(x=x.to(DEV), edge_index=ei.to(DEV), edge_attr=ea.to(DEV)))
    (y * gy.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    print(f"iter {it}: y rel {((y.double().cpu() - y64).norm() / y64.norm()).item():.2e}")
    for k, p in mod.named_parameters():
        d = p.grad.double().cpu() - p64[k].grad
        e = (d.norm() / p64[k].grad.norm()).item()
        if e > 1e-5 or k.startswith("nodes_encoder"):
            am = d.abs().argmax().item()
            print(f"  {k:40s} {e:.2e} max|d| {d.abs().max().item():.2e} at {divmod(am, p.shape[-1]) if p.dim() == 2 else am}")
