"""Bitwise A/B of two libmgn builds: one EncodeProcessDecode forward + backward per config with the
library at argv[1] (a path: swapped into graphphysics._native.LIB_PATH), outputs saved to argv[2];
with argv[3] (an earlier output file) every tensor is compared bit for bit.
    python tools/dev/cmp_libs.py <lib.so> <out.pt> [<ref.pt>]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]
from graphphysics import _native  # noqa: E402

_native.LIB_PATH = os.path.abspath(sys.argv[1])
from graphphysics.models.processors import EncodeProcessDecode  # noqa: E402
from graphphysics.utils import meshes  # noqa: E402
from graphphysics.utils.data import Data  # noqa: E402

DEV = torch.device("cuda:0")
CFGS = [("A_fp32_h32", 5, 32, torch.float32, 1), ("C_bf16_h64", 4, 64, torch.bfloat16, 1),
        ("fp32_h64", 3, 64, torch.float32, 2), ("bf16_h32", 3, 32, torch.bfloat16, 1),
        ("B_bf16_h128", 4, 128, torch.bfloat16, 8), ("fp32_h128", 3, 128, torch.float32, 2),
        ("bf16_h16", 3, 16, torch.bfloat16, 1)]
out = {}
for name, mp, h, dt, batch in CFGS:
    b = meshes.cylinder_batch(batch, jitter=0.01)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(b["x"].shape[0], 11, generator=g).to(DEV).requires_grad_(True)
    ea = torch.from_numpy(b["edge_attr"]).to(DEV).requires_grad_(True)
    d = Data(x=x, edge_index=torch.from_numpy(b["edge_index"]).to(DEV), edge_attr=ea)
    torch.manual_seed(0)
    m = EncodeProcessDecode(mp, 11, 3, 2, h, compute_dtype=dt).to(DEV)
    y = m(d)
    y.backward(torch.randn(y.shape, generator=g).to(DEV))
    torch.cuda.synchronize()
    out[name] = [y.detach().cpu(), x.grad.cpu(), ea.grad.cpu()] + [p.grad.cpu() for p in m.parameters()]
torch.save(out, sys.argv[2])
if len(sys.argv) > 3:
    ref = torch.load(sys.argv[3])
    bad = 0
    for k, ts in out.items():
        for i, (a, c) in enumerate(zip(ts, ref[k])):
            if not torch.equal(a, c):
                bad += 1
                print("DIFF", k, i, float((a - c).abs().max()))
    print("bitwise", "identical" if bad == 0 else f"{bad} tensors differ")
