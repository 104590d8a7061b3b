"""Diagnostic: time the fused edge-MLP forward kernel with phases removed (MGN_ABLATE bits:
1 gather, 2 R8 saves, 4 MFMA, 8 epilogue stores). Cfg B block shapes, bf16."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
import torch
import __graft_entry__ as ge
ge.build()
from graphphysics import _native as nat
from graphphysics.models.layers import GraphNetBlock
from graphphysics.utils import meshes
dev = torch.device("cuda:0")
b = meshes.cylinder_batch(8, jitter=0.01)
ei = torch.from_numpy(b["edge_index"]).to(dev)
N, E, h = b["x"].shape[0], ei.shape[1], 128
torch.manual_seed(0)
blk = GraphNetBlock(h); blk.compute_dtype = torch.bfloat16; blk = blk.to(dev)
x = torch.randn(N, h, device=dev); e = torch.randn(E, h, device=dev)
for mask in (0, 1, 2, 4, 8, 2 | 8, 1 | 2 | 8, 1 | 2 | 4 | 8, 4 | 2):
    os.environ["MGN_ABLATE"] = str(mask)
    with torch.no_grad():
        for _ in range(3):
            blk(x, ei, e)
        torch.cuda.synchronize()
        nat.profile_enable(True)
        for _ in range(10):
            blk(x, ei, e)
        torch.cuda.synchronize()
        p = nat.profile_collect()
        nat.profile_enable(False)
    fe, fn = p["fwd_edge"], p["fwd_node"]
    print(f"ablate={mask:2d}  fwd_edge {1000*fe[0]/max(fe[1],1):7.1f} us   fwd_node {1000*fn[0]/max(fn[1],1):7.1f} us")
