"""Spread of per-wave start / end times inside one launch of each chained kernel kind (MGN_STAMPS
builds: mgn_debug_wave_times). One eager Cfg B training step (bf16, MP=15, h=128, batch 8), then the
last launch of each kind: quantiles of wave start and end relative to the earliest start, in us."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]
from graphphysics import _native as nat  # noqa: E402
from graphphysics.models.processors import EncodeProcessDecode  # noqa: E402
from graphphysics.utils import meshes  # noqa: E402
from graphphysics.utils.data import Data  # noqa: E402

dev = torch.device("cuda:0")
b = meshes.cylinder_batch(8, jitter=0.01)
d = Data(x=torch.randn(b["x"].shape[0], 11, device=dev), edge_index=torch.from_numpy(b["edge_index"]).to(dev),
         edge_attr=torch.from_numpy(b["edge_attr"]).to(dev))
m = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16).to(dev)
for _ in range(3):
    y = m(d)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
L = nat.lib()
for kind, name in enumerate(("edge fwd", "edge bwd", "node fwd", "node bwd")):
    buf = np.zeros((4096, 2), dtype=np.uint64)
    rc = L.mgn_debug_wave_times(kind, ctypes.c_void_p(buf.ctypes.data), 4096)
    assert rc == 0, rc
    v = buf[(buf[:, 0] > 0) & (buf[:, 1] >= buf[:, 0])].astype(np.int64)
    t0 = v[:, 0].min()
    st, en = (v[:, 0] - t0) / 100.0, (v[:, 1] - t0) / 100.0
    q = lambda a: " ".join("%.1f" % x for x in np.quantile(a, [0, 0.1, 0.5, 0.9, 0.99, 1.0]))  # noqa: E731
    print(f"{name:9s} waves {len(v):5d}  start us q0/10/50/90/99/100: {q(st)}  end: {q(en)}")
