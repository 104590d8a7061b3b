"""Experiment: intra-GPU data parallelism. Two half-batches (4 CylinderFlow graphs each) trained by two
captured TrainSteps replayed CONCURRENTLY on two streams, persistent grids capped at MGN_MAX_CUS CUs
each, vs one full-batch (8 graphs) step. Prints the equivalent full-batch steps/s of each.
    MGN_MAX_CUS=128 python tools/exp_dual.py dual      (two half-batch steps on two streams)
    python tools/exp_dual.py single                    (the bench step)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]


def make(batch, seed):
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.optim import FusedAdamW
    from graphphysics.training.step import TrainStep
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data
    from graphphysics.utils.scheduler import CosineWarmupScheduler

    dev = torch.device("cuda:0")
    b = meshes.cylinder_batch(batch, t=0, jitter=0.01, seed=seed)
    data = Data(**{k: torch.from_numpy(b[k]).to(dev) for k in ("x", "y", "edge_index", "edge_attr")})
    torch.manual_seed(0)
    m = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16)
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, m, dev)
    opt = FusedAdamW(sim.parameters(), lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.95))
    sch = CosineWarmupScheduler(opt, warmup=1000, max_iters=10 ** 6)
    st = TrainStep(sim, opt, sch, data, graph=True)
    st.capture(warmup=2)
    return st


def main():
    import __graft_entry__ as ge

    ge.build()
    mode = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    if mode == "single":
        st = make(8, 1234)
        for _ in range(20):
            st()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            st()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"single full-batch: {n / dt:.1f} steps/s ({1e3 * dt / n:.3f} ms/step)")
        return
    a, b = make(4, 1234), make(4, 99)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for s in (a, b):
        s()
    torch.cuda.synchronize()

    def pair():
        a.opt.stage()
        b.opt.stage()
        cur = torch.cuda.current_stream()
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        with torch.cuda.stream(sa):
            a.graph.replay()
        with torch.cuda.stream(sb):
            b.graph.replay()
        cur.wait_stream(sa)
        cur.wait_stream(sb)
        a.sched.step()
        b.sched.step()

    for _ in range(20):
        pair()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        pair()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"dual half-batch (MGN_MAX_CUS={os.environ.get('MGN_MAX_CUS')}): {n / dt:.1f} full-batch-equivalent "
          f"steps/s ({1e3 * dt / n:.3f} ms per pair)")
    # each alone, for reference
    t0 = time.perf_counter()
    for _ in range(n):
        a()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"one half-batch alone: {1e3 * dt / n:.3f} ms/step")


if __name__ == "__main__":
    main()
