"""bench.py — training-steps/sec of the MeshGraphNet hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N)

Workload (BASELINE.json configs[1], SURVEY.md §8d Cfg B): CylinderFlow MeshGraphNet, 15 message-passing
blocks, hidden 128, batch = 8 graphs per GPU (8 jittered copies of the reference's in-tree CylinderFlow
mesh: N=15,384 nodes, E=88,560 edges per GPU), random-init weights (torch.manual_seed(0)), synthetic
velocity frames from the same mesh. One step = Simulator train-mode preamble (3 online normalizers,
one-hot) → EncodeProcessDecode forward → masked L2 loss → backward → [RCCL gradient all-reduce] →
AdamW(wd 1e-4, β (0.9, 0.95)) → cosine-warmup LR step, exactly the reference training_step
(lightning_module.py:111-122, 275-292). Inputs are resident in HBM before timing starts.

value = (steps completed by all ranks) / (max-over-ranks wall time of the K timed steps); each rank's
step is one batch-8 CylinderFlow step, so value/N is the per-GPU step rate (weak scaling).
Extra JSON fields: roofline (dominant kernel, HIP-event timed over the timed region), cpu_baseline
(reference-semantics CPU path = oracle, timed on this host's cores, rank 0, N=1), one_step_mse
(GPU vs reference CPU path on held-out frames with the trained weights), kernels (per-class times).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]

METRIC = "training-steps/sec + one-step velocity MSE, CylinderFlow MGN 15MP h=128"
PEAK = {"bf16": 2500.0, "fp32": 157.3}  # TFLOP/s dense (MI355X_MICROARCH.md)
HBM_PEAK = 8000.0  # GB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="graphs per GPU")
    ap.add_argument("--mp", type=int, default=15)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-steps", type=int, default=2, help="timed CPU baseline steps (0: skip)")
    ap.add_argument("--no-mse", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of hipGraph replay")
    ap.add_argument("--dp", action="store_true",
                    help="use the data-parallel step (exchanges + split graph) even on one rank")
    ap.add_argument("--workload", default="cylinder", choices=["cylinder", "aneurysm"],
                    help="cylinder: Cfg B (headline); aneurysm: Cfg E (1 k-hop-2 aneurysm graph per GPU)")
    return ap.parse_args()


def make_workload(a, dev, rank, mesh):
    """Host arrays + device Data + Simulator layout of the benchmarked configuration.
    cylinder (Cfg B, BASELINE.json configs[1]): a.batch jittered copies of the CylinderFlow mesh.
    aneurysm (Cfg E, configs[4] per GPU): the reference's 3D aneurysm mock mesh (N=22,535,
    115,275 tetrahedra), graph built ON DEVICE by libmgn (FaceToEdge → k-hop 2 → Cartesian +
    Distance: E=1,395,256, max in-degree 103), synthetic node features (14 channels + node type),
    Simulator layout of coarse-aneurysm.json (features 0:14, outputs 0:3, type at 14)."""
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    if a.workload == "cylinder":
        b = meshes.cylinder_batch(a.batch, t=0, jitter=0.01, seed=1234 + rank, mesh=mesh)
        data = Data(x=torch.from_numpy(b["x"]).to(dev), y=torch.from_numpy(b["y"]).to(dev),
                    edge_index=torch.from_numpy(b["edge_index"]).to(dev),
                    edge_attr=torch.from_numpy(b["edge_attr"]).to(dev), pos=torch.from_numpy(b["pos"]).to(dev))
        return b, data, dict(node_in=11, edge_in=3, out=2, fs=(0, 2), os=(0, 2), nti=2), \
            "CylinderFlow MGN %dMP h=%d, batch=%d graphs per GPU (Cfg B)" % (a.mp, a.hidden, a.batch), \
            "%d jittered copies of the reference in-tree CylinderFlow mesh per GPU" % a.batch
    from graphphysics.utils import graph_build as G

    z = np.load(os.path.join(ROOT, "tests", "golden", "aneurysm_mesh.npz"))
    pos = torch.from_numpy(z["pos"]).to(dev)
    tet = torch.from_numpy(z["tetra"].astype(np.int64)).t().contiguous().to(dev)
    n = pos.shape[0]
    ei = G.k_hop_edge_index(G.face_to_edge(tet, n), 2, n)
    ea = G.edge_features(pos, ei)
    rng = np.random.default_rng(1234 + rank)
    feats = rng.standard_normal((n, 14)).astype(np.float32)
    nt = rng.choice([0, 4, 5, 6], size=n, p=[0.9, 0.01, 0.01, 0.08]).astype(np.float32)
    x = np.concatenate([feats, nt[:, None]], 1)
    y = (feats[:, 0:3] + 0.01 * rng.standard_normal((n, 3))).astype(np.float32)
    data = Data(x=torch.from_numpy(x).to(dev), y=torch.from_numpy(y).to(dev), edge_index=ei, edge_attr=ea, pos=pos)
    b = {"x": x, "y": y, "edge_index": ei.cpu().numpy(), "edge_attr": ea.cpu().numpy()}
    return b, data, dict(node_in=23, edge_in=4, out=3, fs=(0, 14), os=(0, 3), nti=14), \
        "3D-CoarseAneurysm MGN %dMP h=%d, 1 graph per GPU, k-hop 2 (Cfg E)" % (a.mp, a.hidden), \
        "reference aneurysm mock mesh (k-hop 2 built on device), synthetic node features"


def flops_per_block(n, e, h):
    # MFMA FLOPs per launch (2·Σ in·out per row). The edge MLP's layer 0 runs on the e block only
    # (the x blocks are applied per node: node_proj / node_grad kernels), so 4 128x128 Linears.
    return 8 * h * h * e, 10 * h * h * n  # edge MLP, node MLP


def bytes_per_block(n, e, h, es):
    """Compulsory HBM bytes per launch of the block kernels (SURVEY §8d unit = one edge / node):
    every input read once, every output written once, gathered rows counted once per use at their
    stored size; es = activation element size (2 bf16, 4 fp32)."""
    mask = 3 * h // 8  # ReLU bits of the 3 hidden layers
    edge_fwd = e * (es * h + es * h * 2 + 3 * es * h + mask + 4 + 2 * 4 * h)
    # e in | out, z | R8 inputs of layers 1..3 | masks | rden | fp32 node projections P_i, P_j gathered
    edge_bwd = e * (3 * es * h + 4 + mask + 3 * es * h + 2 * es * h)
    # de_out, d_aggr[dst], z in | rden | masks | dZ of layers 1..3 (R8) | de, dZ0 row-major out
    node_fwd = e * (es * h + 4) + n * (es * h + 3 * es * h + 4 + mask + 3 * es * h)
    # edge z + rden (segment sum) | x in; x_out, aggr, z out; rden; masks; R8 inputs of layers 1..3
    node_bwd = n * (es * h + es * h + 4 + mask + 4 * es * h + 2 * es * h)
    # dx_out, z in | rden | masks | dZ of 4 layers (R8) | dx_part, d_aggr out
    return {"fwd_edge": edge_fwd, "bwd_edge": edge_bwd, "fwd_node": node_fwd, "bwd_node": node_bwd}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != a.gpus:
        a.gpus = world
    # MGN_DIST_BACKEND=gloo (rehearsal only): several ranks share the visible GPUs round-robin and
    # exchange through host memory; the default "nccl" is RCCL over xGMI, one rank per GPU
    backend = os.environ.get("MGN_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or a.dp:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)  # RCCL over xGMI
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    import __graft_entry__ as ge

    if rank == 0:
        ge.build()
    if world > 1:
        dist.barrier()
    ge._paths()
    from graphphysics import _native as nat
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.optim import FusedAdamW
    from graphphysics.training.step import TrainStep
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data
    from graphphysics.utils.nodetype import NodeType
    from graphphysics.utils.scheduler import CosineWarmupScheduler

    nat.load()
    cdt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    mesh = meshes.load_cylinder_mesh()
    b, data, lay, workload, datadesc = make_workload(a, dev, rank, mesh)
    N, E = data.x.shape[0], data.edge_index.shape[1]
    torch.manual_seed(0)
    model = EncodeProcessDecode(a.mp, lay["node_in"], lay["edge_in"], lay["out"], a.hidden, compute_dtype=cdt)
    sim = Simulator(lay["node_in"], lay["edge_in"], lay["out"], lay["fs"][0], lay["fs"][1], lay["os"][0],
                    lay["os"][1], lay["nti"], model, dev)
    params = list(sim.parameters())
    opt = FusedAdamW(params, lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.95))
    sched = CosineWarmupScheduler(opt, warmup=1000, max_iters=10 ** 6)
    sim.train()
    step = TrainStep(sim, opt, sched, data, graph=not a.no_graph, data_parallel=(world > 1 or a.dp))
    if step.use_graph:
        step.capture(warmup=max(a.warmup - 1, 1))
        step()  # first replay
    else:
        for _ in range(a.warmup):
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    prof = {}
    if not a.no_profile:
        # Per-kernel durations: HIP events on the launch stream around every kernel of K more steps
        # run eagerly (the same kernels, shapes and launch order the replayed graph contains).
        nat.profile_enable(True)
        for _ in range(a.steps):
            step.eager()
        torch.cuda.synchronize()
        prof = nat.profile_collect()
        nat.profile_enable(False)
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    last_loss = float(loss.item())

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    h = a.hidden
    fe, fn = flops_per_block(N, E, h)
    alg_bytes = bytes_per_block(N, E, h, 2 if a.dtype == "bf16" else 4)
    kinds = {}
    for k, (ms, cnt) in prof.items():
        if cnt:
            kinds[k] = {"total_ms": round(ms, 4), "launches": cnt, "avg_us": round(1000 * ms / cnt, 2)}
    # algorithmic work per launch of each kernel class: MFMA FLOPs
    alg_flops = {"fwd_edge": fe, "fwd_node": fn, "bwd_edge": fe, "bwd_node": fn}
    roof = None
    if kinds:
        dom = max((k for k in kinds if k in alg_flops), key=lambda k: kinds[k]["total_ms"])
        avg_s = kinds[dom]["total_ms"] / 1000 / kinds[dom]["launches"]
        tf = alg_flops[dom] / avg_s / 1e12
        gbs = alg_bytes[dom] / avg_s / 1e9
        mfma = {"achieved": round(tf, 2), "peak": PEAK[a.dtype], "unit": "TFLOP/s", "frac": round(tf / PEAK[a.dtype], 4)}
        hbm = {"achieved": round(gbs, 1), "peak": HBM_PEAK, "unit": "GB/s", "frac": round(gbs / HBM_PEAK, 4)}
        bound = "hbm" if hbm["frac"] >= mfma["frac"] else "mfma"
        roof = {"kernel": dom, "bound": bound, **(hbm if bound == "hbm" else mfma), "traffic": None,
                "bytes_per_launch": alg_bytes[dom], "flops_per_launch": alg_flops[dom],
                "avg_launch_us": round(avg_s * 1e6, 2), "hbm": hbm, "mfma": mfma}
        step_flops = 3 * (a.mp * (fe + fn) + 2 * (lay["edge_in"] * h + 3 * h * h) * E
                          + 2 * (lay["node_in"] * h + 3 * h * h) * N + 2 * (3 * h * h + h * lay["out"]) * N)
        roof["step_tflops_per_s"] = round(step_flops * a.steps / dt / 1e12, 2)
    if roof is not None:
        roof["traffic"], roof["traffic_note"] = pmc_traffic(roof["kernel"])
    value = world * a.steps / dt
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
        "data": "synthetic: %s, random-init weights (seed 0)" % datadesc,
        "execution": ("eager" if not step.use_graph else
                      "hipGraph replay of forward+loss+backward; eager statistics/gradient all-reduce + AdamW"
                      if step.dp else "hipGraph replay of the whole step"),
        "config": {"workload": workload, "nodes_per_gpu": N, "edges_per_gpu": E,
                   "global_batch": (a.batch if a.workload == "cylinder" else 1) * world,
                   "parallelism": "dp%d" % world,
                   "graphs_per_sec": round(value * (a.batch if a.workload == "cylinder" else 1), 2)},
        "roofline": roof, "kernels": kinds, "last_loss": last_loss,
    }

    if not a.no_mse and a.workload == "cylinder":
        out["one_step_mse"] = one_step_mse(sim, mesh, dev, a)
    if world == 1 and a.cpu_steps > 0:
        out["cpu_baseline"] = cpu_baseline(a, b, lay)
        if out["cpu_baseline"]:
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


def pmc_traffic(kernel_class):
    """HBM bytes per launch of `kernel_class` from the committed rocprofv3 PMC passes
    (profiles/<round>_traffic.json, made by tools/profile_round.sh + tools/pmc_traffic.py), used only
    when they were measured on the same kernel sources (sha256 stamp)."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import sources_sha

    sha = sources_sha()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        d = json.load(open(f))
        if d.get("sources_sha") == sha and kernel_class in d.get("kernels", {}):
            return round(d["kernels"][kernel_class]["hbm_bytes"]), os.path.relpath(f, ROOT)
    return None, "no PMC traffic measured for these kernel sources (run tools/profile_round.sh)"


def one_step_mse(sim, mesh, dev, a):
    """Held-out CylinderFlow frames 3→4 and 4→5 (B=1): eval-mode prediction with the trained weights
    through libmgn vs through the reference-semantics CPU path (oracle, fp32) with the same weights
    and normalizer statistics; masked MSE as the reference val_loss (lightning_module.py:168-232)."""
    from oracle import mgn_oracle as O
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    sim.eval()
    ref = O.OracleEPD(a.mp, 11, 3, 2, a.hidden)
    ref.load_state_dict({k: v.detach().float().cpu() for k, v in sim.model.state_dict().items()})
    osim = O.OracleSimulator(ref, 11, 3, 2)
    for mine, theirs in ((sim._output_normalizer, osim.out_norm), (sim._node_normalizer, osim.node_norm),
                         (sim._edge_normalizer, osim.edge_norm)):
        theirs.acc_sum = mine._acc_sum.detach().cpu().clone()
        theirs.acc_sum_squared = mine._acc_sum_squared.detach().cpu().clone()
        theirs.acc_count = mine._acc_count.detach().cpu().clone()
        theirs.num_acc = mine._num_accumulations.detach().cpu().clone()
    gm, rm = [], []
    for t in (3, 4):
        bb = meshes.cylinder_batch(1, t=t, mesh=mesh)
        x, y = torch.from_numpy(bb["x"]), torch.from_numpy(bb["y"])
        ei, ea = torch.from_numpy(bb["edge_index"]), torch.from_numpy(bb["edge_attr"])
        nt = x[:, 2]
        keep = ~((nt == 0) | (nt == 5))
        with torch.no_grad():
            _, _, pred = sim(Data(x=x.to(dev), y=y.to(dev), edge_index=ei.to(dev), edge_attr=ea.to(dev)))
            pred = pred.cpu()
            _, _, pr = osim.forward(x, y, ei, ea, training=False)
        pred[keep], pr[keep] = y[keep], y[keep]
        gm.append(O.l2_loss(y, pred, nt).item())
        rm.append(O.l2_loss(y, pr, nt).item())
    sim.train()
    g, r = float(np.mean(gm)), float(np.mean(rm))
    return {"gpu": g, "reference_cpu": r, "abs_diff": abs(g - r), "target_abs_diff": 1e-5,
            "frames": "3->4, 4->5 (held out), B=1, weights after the timed steps"}


def cpu_baseline(a, b, lay):
    """The reference algorithm on the host (oracle = op-for-op restatement of the reference's
    PyTorch CPU path, pinned to golden vectors), same workload (Cfg B batch 8), fp32, all cores."""
    from oracle import mgn_oracle as O

    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    ref = O.OracleEPD(a.mp, lay["node_in"], lay["edge_in"], lay["out"], a.hidden)
    osim = O.OracleSimulator(ref, lay["node_in"], lay["edge_in"], lay["out"], feature_slice=lay["fs"],
                             output_slice=lay["os"], node_type_index=lay["nti"])
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.95))
    x, y = torch.from_numpy(b["x"]), torch.from_numpy(b["y"])
    ei, ea = torch.from_numpy(b["edge_index"]), torch.from_numpy(b["edge_attr"])

    def step():
        opt.zero_grad()
        net, tdn, _ = osim.forward(x, y, ei, ea, True)
        O.l2_loss(tdn, net, x[:, lay["nti"]]).backward()
        opt.step()

    step()  # warm-up
    ts = []
    for _ in range(a.cpu_steps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    med = float(np.median(ts))
    import platform

    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(1.0 / med, 4), "unit": "steps/s", "cores": cores, "kind": "port",
            "sample": "%d timed + 1 warm-up full steps of the same workload (N=%d, E=%d), torch %s fp32, median"
                      % (a.cpu_steps, b["x"].shape[0], b["edge_index"].shape[1], torch.__version__),
            "cpu": model, "host": platform.node()}


if __name__ == "__main__":
    main()
