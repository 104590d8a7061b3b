"""Diagnostic: train the bench model a few captured steps and report non-finite parameters,
gradients or buffers (per tensor, with the first bad index)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "graph-physics_amd")]
import torch  # noqa: E402

import __graft_entry__ as ge  # noqa: E402

ge.build()
from graphphysics.models.processors import EncodeProcessDecode  # noqa: E402
from graphphysics.models.simulator import Simulator  # noqa: E402
from graphphysics.training.optim import FusedAdamW  # noqa: E402
from graphphysics.training.step import TrainStep  # noqa: E402
from graphphysics.utils import meshes  # noqa: E402
from graphphysics.utils.data import Data  # noqa: E402
from graphphysics.utils.scheduler import CosineWarmupScheduler  # noqa: E402

dev = torch.device("cuda:0")
b = meshes.cylinder_batch(8, t=0, jitter=0.01, seed=1234)
data = Data(**{k: torch.from_numpy(b[k]).to(dev) for k in ("x", "y", "edge_index", "edge_attr", "pos")})
torch.manual_seed(0)
model = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16)
sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, model, dev)
opt = FusedAdamW(list(sim.parameters()), lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.95))
sched = CosineWarmupScheduler(opt, warmup=1000, max_iters=10 ** 6)
sim.train()
step = TrainStep(sim, opt, sched, data, graph=True)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    loss = step()
    torch.cuda.synchronize()
    bad = []
    for k, p in sim.named_parameters():
        for tag, t in (("param", p), ("grad", p.grad)):
            if t is not None and not torch.isfinite(t).all():
                idx = (~torch.isfinite(t)).nonzero()[:3].tolist()
                bad.append(f"{tag} {k} {tuple(t.shape)} n={int((~torch.isfinite(t)).sum())} at {idx}")
    for k, t in sim.named_buffers():
        if not torch.isfinite(t).all():
            bad.append(f"buffer {k}")
    print(f"step {i} loss {float(loss.detach()):.4f} nonfinite: {len(bad)}", flush=True)
    for line in bad[:12]:
        print("   ", line, flush=True)
