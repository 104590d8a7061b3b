"""Diagnostics: where does the data-parallel step's time go? Times each phase of
TrainStep.__call__ (dp mode) separately over K repetitions on a 1-rank process group.
python tools/dp_phases.py [--backend nccl|gloo]"""
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]


def main():
    backend = sys.argv[sys.argv.index("--backend") + 1] if "--backend" in sys.argv else "nccl"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29512")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    else:
        dist.init_process_group(backend, rank=0, world_size=1)
    import __graft_entry__ as ge

    ge.build()
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.distributed import allreduce_gradients
    from graphphysics.training.optim import FusedAdamW
    from graphphysics.training.step import TrainStep
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data
    from graphphysics.utils.scheduler import CosineWarmupScheduler

    b = meshes.cylinder_batch(8, t=0, jitter=0.01, seed=1234)
    data = Data(x=torch.from_numpy(b["x"]).to(dev), y=torch.from_numpy(b["y"]).to(dev),
                edge_index=torch.from_numpy(b["edge_index"]).to(dev),
                edge_attr=torch.from_numpy(b["edge_attr"]).to(dev))
    torch.manual_seed(0)
    model = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16)
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, model, dev)
    opt = FusedAdamW(list(sim.parameters()), lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.95))
    sched = CosineWarmupScheduler(opt, warmup=1000, max_iters=10 ** 6)
    sim.train()
    step = TrainStep(sim, opt, sched, data, graph=True, data_parallel=True)
    step.capture(warmup=2)
    step()
    torch.cuda.synchronize()
    K = 20

    def timed(name, fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        print("%-28s %8.3f ms/iter (host enqueue %8.3f ms/iter)" % (name, 1e3 * t / K, 1e3 * th / K), flush=True)

    timed("full dp step", step)
    timed("opt.stage", opt.stage)
    timed("prologue (exchange stats)", step._prologue)
    timed("graph replay", step.graph.replay)
    timed("allreduce_gradients", lambda: allreduce_gradients(step.params, step.group))
    timed("opt.launch", opt.launch)
    timed("sched.step", sched.step)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
