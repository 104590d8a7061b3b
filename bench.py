"""bench.py — training-steps/sec of the MeshGraphNet hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    N>1: `python bench.py --gpus N` starts its N ranks itself (torch.distributed.run as a child process,
    before anything touches the GPU) and forwards rank 0's JSON line; run under a launcher
    (python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N) it is
    one of the launcher's ranks.

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

OUT = sys.stdout  # the JSON line's stream (main() keeps the real stdout for it alone)
METRIC = "training-steps/sec + one-step velocity MSE, CylinderFlow MGN 15MP h=128"
PEAK = {"bf16": 2500.0, "fp32": 157.3}  # TFLOP/s dense (MI355X_MICROARCH.md)
HBM_PEAK = 8000.0  # GB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps (0.3 s at Cfg B) after 20 warm-up replays: a 20-step window carried ~1.6 % of fixed
    # start-up cost (same box: 343.9 -> 349.6 steps/s, tools/dev/r06_steps.sh)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8, help="graphs per GPU")
    ap.add_argument("--mp", type=int, default=15)
    ap.add_argument("--hidden", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-steps", type=int, default=10,
                    help="timed CPU baseline steps after 3 warm-up steps (SURVEY §8(d): >= 10 timed, 3 warm-up; "
                         "a bounded sample, ~100 s on 16 cores) of the same workload, median reported (0: skip)")
    ap.add_argument("--sustain", type=float, default=5.0,
                    help="seconds of further replayed steps after the timed K (reported as `sustained`)")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the Config B fp32 and Config A rows (N=1 only)")
    ap.add_argument("--no-mse", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of hipGraph replay")
    ap.add_argument("--fresh-batch", action="store_true",
                    help="eager steps on a NEW batch each step (fresh device copies of x / y / edge_index / "
                         "edge_attr, so the topology is rebuilt): the Lightning Trainer path "
                         "(reference train.py:233-262 collates a new Batch per step); implies --no-graph")
    ap.add_argument("--dp", action="store_true",
                    help="use the data-parallel step (exchanges + split graph) even on one rank")
    ap.add_argument("--workload", default="cylinder", choices=["cylinder", "aneurysm", "plate"],
                    help="cylinder: Cfg B (headline); aneurysm: Cfg E (1 k-hop-2 aneurysm graph per GPU); "
                         "plate: Cfg C (DeformingPlate-shaped tet mesh + world edges)")
    ap.add_argument("--print-workload", action="store_true",
                    help="print the workload key the PMC files are stamped with, and exit")
    ap.add_argument("--dry", action="store_true",
                    help="launcher check: start the ranks, form the process group (gloo), agree on the world "
                         "size, print the JSON line's rank/world fields and exit before any GPU call")
    a = ap.parse_args()
    if a.fresh_batch:
        a.no_graph = True
    return a


def workload_key(a):
    """Stamp of the measured configuration (PMC files only apply to the same one)."""
    return "%s:b%d:mp%d:h%d:%s" % (a.workload, a.batch if a.workload == "cylinder" else 1, a.mp, a.hidden, a.dtype)


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
            "CylinderFlow MGN %dMP h=%d, batch=%d graphs per GPU (%s)" % (
                a.mp, a.hidden, a.batch, "Cfg B" if (a.mp, a.hidden, a.batch) == (15, 128, 8) else
                "Cfg A" if (a.mp, a.hidden, a.batch) == (5, 32, 1) else "custom"), \
            "%d jittered copies of the reference in-tree CylinderFlow mesh per GPU" % a.batch
    if a.workload == "plate":
        g, lay = meshes.plate_graph(dev, seed=rank)
        b = {"x": g.x.cpu().numpy(), "y": g.y.cpu().numpy(), "edge_index": g.edge_index.cpu().numpy(),
             "edge_attr": g.edge_attr.cpu().numpy()}
        data = Data(x=g.x, y=g.y, edge_index=g.edge_index, edge_attr=g.edge_attr, pos=g.pos)
        return b, data, lay, "DeformingPlate MGN %dMP h=%d, 1 graph per GPU, world edges (Cfg C)" % (a.mp, a.hidden), \
            "DeformingPlate-shaped tet plate + obstacle (meshes.plate_sample), reference preprocessing on device"
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


def class_work(n, e, h, mp, lay, nparams, nweights, es, launches=None):
    """Work per STEP of every kernel class: {class: (bound, executed, algorithmic)}, FLOPs for "mfma"
    classes, bytes for "hbm" ones (SURVEY.md §8(a,d) per-unit figures x the units the class processes).
    `executed` is what the class's kernels compute: the per-class `frac` uses it, so no class is credited
    with work another class (or no kernel) does. `algorithmic` is the reference algorithm's work the
    class stands for (§8(d)): reported beside the executed figure for the dominant class only.
      edge layer 0 is split: fwd_edge runs the e block + 3 hidden Linears (8h²/edge); the
      x_i / x_j blocks become node projections, 4h²/NODE, in `proj` (one launch per block on the
      generic path, block 0 only on the chained bf16 path) or inside the previous block's node-MLP
      forward (chained hand-off); bwd_edge 8h²/edge; combine (node_grad) dx += [dP_i‖dP_j]·W0[:, h:3h]ᵀ,
      4h²/node; node MLP 10h²/node fwd and bwd; weight gradients (ring, or the generic kernel on the
      generic path) 8h²/edge + 14h²/node executed vs the reference's 12h²/edge + 10h²/node;
      encoders/decoder 2(in·h + 3h²) per row fwd and weight gradients, backward data 6h² per encoder
      row (no input gradient) + the decoder's 2(3h² + h·out). AdamW: p, g, m, v read + p, m, v
      written (28 B/param); pack: fp32 weights in, 2 bf16 copies out."""
    launches = launches or {}
    enc = 2 * (lay["edge_in"] * h + 3 * h * h) * e + 2 * (lay["node_in"] * h + 3 * h * h) * n
    dec = 2 * (3 * h * h + h * lay["out"]) * n
    nproj = launches.get("proj", mp)  # projection launches per step
    handoff = max(mp - nproj, 0)      # blocks whose projections run inside the previous node-MLP forward
    wg_exec, wg_alg = mp * (8 * h * h * e + 14 * h * h * n), mp * (12 * h * h * e + 10 * h * h * n)
    return {
        "fwd_edge": ("mfma", mp * 8 * h * h * e, mp * 12 * h * h * e),
        "proj": ("mfma", nproj * 4 * h * h * n, None),
        "fwd_node": ("mfma", mp * 10 * h * h * n + handoff * 4 * h * h * n, mp * 10 * h * h * n),
        "bwd_edge": ("mfma", mp * 8 * h * h * e, mp * 12 * h * h * e),
        "combine": ("mfma", mp * 4 * h * h * n, None),
        "bwd_node": ("mfma", mp * 10 * h * h * n, mp * 10 * h * h * n),
        "wgrad": ("mfma", wg_exec, wg_alg),
        "fwd_dense": ("mfma", enc + dec, enc + dec),
        "bwd_dense": ("mfma", 6 * h * h * (e + n) + dec, enc + dec),
        "wgrad_dense": ("mfma", enc + dec, enc + dec),
        "adamw": ("hbm", 28 * nparams, 28 * nparams), "pack": ("hbm", 8 * nweights, 8 * nweights),
    }


def scatter_bytes(n, e, h, es):
    """SURVEY §8(a5,d): segmented-sum bytes per block forward, E·h·s + N·h·s + 4E + 4(N+1)."""
    return e * h * es + n * h * es + 4 * e + 4 * (n + 1)


def scatter_standalone(a, data, dev):
    """The same segmented sum as a kernel of its own (`mgn_segment_sum`, the ABI's scatter_add
    replacement: one thread per segment and 16-byte chunk, rows read in CSC order) over the step's
    topology and an [E, h] message tensor of the compute dtype: HIP-event time of 50 launches."""
    from graphphysics import _native as nat
    from graphphysics.models import _engine

    N, E, h = data.x.shape[0], data.edge_index.shape[1], a.hidden
    tdt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    topo = _engine.get_topology(data.edge_index, N)
    z = torch.randn(E, h, device=dev).to(tdt)
    out = torch.empty(N, h, device=dev, dtype=tdt)
    mdt = nat.MGN_BF16 if a.dtype == "bf16" else nat.MGN_F32
    st = nat.stream_ptr(dev)

    def run():
        nat.check(nat.lib().mgn_segment_sum(nat.ptr(z), nat.ptr(topo.col_ptr), N, h, mdt, nat.ptr(out), st))

    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        run()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1000 / 50
    sb = scatter_bytes(N, E, h, 2 if a.dtype == "bf16" else 4)
    return {"kernel": "mgn_segment_sum (standalone, same topology and sizes)", "bytes_per_launch": sb,
            "avg_launch_us": round(t * 1e6, 2), "achieved": round(sb / t / 1e9, 1), "peak": HBM_PEAK, "unit": "GB/s",
            "frac": round(sb / t / 1e9 / HBM_PEAK, 4)}


def build_step(a, dev, rank, mesh, world):
    """Workload + Simulator + FusedAdamW + schedule + TrainStep of configuration `a`."""
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.optim import FusedAdamW
    from graphphysics.training.step import TrainStep
    from graphphysics.utils.scheduler import CosineWarmupScheduler

    cdt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    b, data, lay, workload, datadesc = make_workload(a, dev, rank, mesh)
    torch.manual_seed(0)
    model = EncodeProcessDecode(a.mp, lay["node_in"], lay["edge_in"], lay["out"], a.hidden, compute_dtype=cdt)
    sim = Simulator(lay["node_in"], lay["edge_in"], lay["out"], lay["fs"][0], lay["fs"][1], lay["os"][0],
                    lay["os"][1], lay["nti"], model, dev)
    opt = FusedAdamW(list(sim.parameters()), lr=1e-3, weight_decay=1e-4, betas=(0.9, 0.95))
    sched = CosineWarmupScheduler(opt, warmup=1000, max_iters=10 ** 6)
    sim.train()
    step = TrainStep(sim, opt, sched, data, graph=not a.no_graph, data_parallel=(world > 1 or a.dp))
    return step, sim, b, data, lay, workload, datadesc


def warm(a, step):
    if step.use_graph:
        step.capture(warmup=max(a.warmup - 1, 1))
        step()  # first replay
    else:
        for _ in range(a.warmup):
            step()
    torch.cuda.synchronize()


PROFILE_SCHEDULE = ("one stream, whole chip: each kernel class timed alone (the timed replay runs the "
                    "processor's weight-gradient launches on a side stream beside the data gradients, each on "
                    "its share of the CUs)")


def profile_classes(a, step):
    """Per-kernel-class durations: HIP events on the launch stream around every kernel of K steps run
    eagerly (the same kernels and shapes the replayed graph contains), after two unprofiled eager steps
    (the first eager step after replays pays one-time costs). On ONE stream (PROFILE_SCHEDULE): a
    kernel's roofline is its own, not its share of a chip it splits with a concurrent launch."""
    from graphphysics import _native as nat
    from graphphysics.models import _engine

    saved = _engine.CONC_WGRAD
    _engine.CONC_WGRAD = "0"
    try:
        for _ in range(2):
            step.eager()
        torch.cuda.synchronize()
        nat.profile_enable(True)
        for _ in range(a.steps):
            step.eager()
        torch.cuda.synchronize()
        prof = nat.profile_collect()
        nat.profile_enable(False)
    finally:
        _engine.CONC_WGRAD = saved
    return prof


def analyse(a, prof, sim, lay, N, E, dt):
    """Per-class work rates and the roofline of the dominant class."""
    h = a.hidden
    es = 2 if a.dtype == "bf16" else 4
    nparams = sum(p.numel() for p in sim.parameters())
    nweights = sum(m.weight.numel() for m in sim.model.modules() if isinstance(m, torch.nn.Linear))
    per_step = {k: cnt / a.steps for k, (ms, cnt) in prof.items() if cnt}
    work = class_work(N, E, h, a.mp, lay, nparams, nweights, es, per_step)
    if not prof.get("wgrad", (0, 0))[1] and prof.get("wgrad_dense", (0, 0))[1]:
        # no ring launches (the generic path): every weight gradient, the processor blocks' too, runs
        # on the generic kernel the profiler files under wgrad_dense
        w, d = work["wgrad"], work["wgrad_dense"]
        work["wgrad_dense"] = ("mfma", w[1] + d[1], w[2] + d[2])
    kinds = {}
    for k, (ms, cnt) in prof.items():
        if cnt:
            kinds[k] = {"total_ms": round(ms, 4), "launches": cnt, "avg_us": round(1000 * ms / cnt, 2),
                        "ms_per_step": round(ms / a.steps, 4)}
            if k in work:
                bound, amount = work[k][:2]
                per_s = amount * a.steps / (ms / 1000)
                if bound == "mfma":
                    kinds[k].update(bound="mfma", tflops=round(per_s / 1e12, 2),
                                    frac=round(per_s / 1e12 / PEAK[a.dtype], 4))
                else:
                    kinds[k].update(bound="hbm", gbs=round(per_s / 1e9, 1), frac=round(per_s / 1e9 / HBM_PEAK, 4))
                if kinds[k]["frac"] > 1.0:  # executed work above peak would be a crediting bug: flagged, not hidden
                    kinds[k]["error"] = "frac above peak: executed-work credit is wrong for this class"
    roof = None
    wl = workload_key(a)
    step_flops = 3 * (a.mp * (12 * h * h * E + 10 * h * h * N) + 2 * (lay["edge_in"] * h + 3 * h * h) * E
                      + 2 * (lay["node_in"] * h + 3 * h * h) * N + 2 * (3 * h * h + h * lay["out"]) * N)
    step_tf = step_flops * a.steps / dt / 1e12
    if kinds:
        # dominant kernel class = largest device time per step of the one-stream per-class profile (each
        # kernel on the whole chip, the launches avg_launch_us times); its share of the
        # REPLAYED step (rocprofv3 kernel trace of this bench command on these sources, recorded with the PMC
        # passes under profiles/, where the ring shares the chip with the data gradients) beside it
        dom = max(kinds, key=lambda k: kinds[k]["total_ms"])
        picked = "one-stream per-class profile (%s)" % ", ".join(
            "%s %.1f us/step" % (k, 1000 * kinds[k]["ms_per_step"])
            for k in sorted(kinds, key=lambda k: -kinds[k]["total_ms"])[:3])
        rep = replay_lookup(wl)
        kd = kinds[dom]
        bound, executed, algorithmic = work.get(dom, ("mfma", 0, None))
        credit = algorithmic if algorithmic is not None else executed
        per_launch = credit * a.steps / kd["launches"]
        per_launch_x = executed * a.steps / kd["launches"]
        avg_s = kd["total_ms"] / 1000 / kd["launches"]
        scale = 1e12 if bound == "mfma" else 1e9
        ach, ach_x = per_launch / avg_s / scale, per_launch_x / avg_s / scale
        peak = PEAK[a.dtype] if bound == "mfma" else HBM_PEAK
        pmc = pmc_lookup(dom, wl)
        unit = "flops" if bound == "mfma" else "bytes"
        in_replay = None
        rr = rep.get("replay", {}).get(dom)
        if rr and rr.get("avg_us"):
            in_replay = {"source": rep["source"], "us_per_step": rr["us_per_step"], "avg_us": rr["avg_us"],
                         "launches_per_step": rr["launches_per_step"],
                         "frac": round(per_launch / (rr["avg_us"] * 1e-6) / scale / peak, 4),
                         "note": "the same work per launch over the class's average launch in the replayed step "
                                 "(concurrent schedule: the ring on its share of the CUs)"}
        roof = {"kernel": dom, "bound": bound, "achieved": round(ach, 2), "peak": peak,
                "unit": "TFLOP/s" if bound == "mfma" else "GB/s", "frac": round(ach / peak, 4),
                "credit": "algorithmic (SURVEY §8(d): the reference algorithm's work this kernel class stands for)"
                          if algorithmic is not None else "executed",
                "executed": {unit + "_per_launch": per_launch_x, "achieved": round(ach_x, 2),
                             "frac": round(ach_x / peak, 4)},
                "traffic": pmc.get("hbm_bytes"), "traffic_source": pmc.get("source"),
                "mfma_util_measured": pmc.get("mfma_util"), "dominant_from": picked,
                "in_replay_frac": in_replay["frac"] if in_replay else None, "in_replay": in_replay,
                "pmc_record": {k: pmc.get(k) for k in ("schedule", "trace_us", "grbm_us_at_2400MHz",
                                                       "implied_clock_mhz", "instances")},
                unit + "_per_launch": per_launch,
                "avg_launch_us": round(avg_s * 1e6, 2), "launches_per_step": kd["launches"] / a.steps,
                "peak_source": "MI355X_MICROARCH.md: dense bf16 MFMA 2.5 PFLOP/s (fp32 MFMA 157.3), HBM3E 8 TB/s",
                "step": {"tflops_per_s": round(step_tf, 2), "frac": round(step_tf / PEAK[a.dtype], 4),
                         "flops_per_step": step_flops, "note": "3 x F_fwd (SURVEY §8d) / measured ms_per_step"}}
        if pmc.get("trace_us"):
            # the PMC record's own launches (rocprofv3 trace of the one-stream run) vs this run's HIP events
            roof["pmc_record"]["trace_us_over_avg_launch_us"] = round(pmc["trace_us"] / (avg_s * 1e6), 3)
        if "fwd_node" in kinds:  # the segmented sum is fused into the node-MLP forward (CSC segments)
            sb = scatter_bytes(N, E, h, es)
            t = kinds["fwd_node"]["total_ms"] / 1000 / kinds["fwd_node"]["launches"]
            roof["scatter"] = {"kernel": "fwd_node (segment sum fused into the node-MLP forward)",
                               "bytes_per_launch": sb, "achieved": round(sb / t / 1e9, 1), "peak": HBM_PEAK,
                               "unit": "GB/s", "frac": round(sb / t / 1e9 / HBM_PEAK, 4)}
        if "combine" in kinds:
            sb = 2 * scatter_bytes(N, E, h, es)
            t = kinds["combine"]["total_ms"] / 1000 / kinds["combine"]["launches"]
            roof["gather_bwd"] = {"kernel": "combine (dP_i / dP_j segment sums over both index directions)",
                                  "bytes_per_launch": sb, "achieved": round(sb / t / 1e9, 1), "peak": HBM_PEAK,
                                  "unit": "GB/s", "frac": round(sb / t / 1e9 / HBM_PEAK, 4)}
    return kinds, roof


def secondary(a0, dev, mesh, label, cpu_steps=0, **over):
    """One more single-GPU configuration timed inside the same invocation (BASELINE.md Config A / B
    rows): warm-up, K timed replayed steps, the eager per-class profile and its roofline, optionally
    the CPU baseline of the same configuration."""
    a = argparse.Namespace(**vars(a0))
    for k, v in over.items():
        setattr(a, k, v)
    step, sim, b, data, lay, workload, datadesc = build_step(a, dev, 0, mesh, 1)
    N, E = data.x.shape[0], data.edge_index.shape[1]
    warm(a, step)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kinds, roof = analyse(a, profile_classes(a, step) if not a.no_profile else {}, sim, lay, N, E, dt)
    r = {"label": label, "workload": workload, "dtype": a.dtype, "mp": a.mp, "hidden": a.hidden,
         "graphs": a.batch, "nodes": N, "edges": E, "steps": a.steps, "value": round(a.steps / dt, 3),
         "unit": "steps/s", "ms_per_step": round(1000 * dt / a.steps, 3),
         "execution": "hipGraph replay of the whole step" if step.use_graph else "eager", "roofline": roof,
         "kernels": {k: {f: v[f] for f in ("avg_us", "ms_per_step", "frac") if f in v} for k, v in kinds.items()}}
    if cpu_steps:
        a.cpu_steps = cpu_steps
        r["cpu_baseline"] = cpu_baseline(a, b, lay, warmup=3)
        r["speedup_vs_cpu"] = round(r["value"] / r["cpu_baseline"]["value"], 1)
    del step, sim, data
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return r


def launch_ranks(a):
    """`python bench.py --gpus N` (N > 1) outside a torch.distributed launcher: start the N ranks as ONE
    child process — torch.distributed.run on this script with the same arguments, one rank per GPU of
    this node, rendezvous on 127.0.0.1 — before this process touches the GPU (no exec: the parent only
    waits). The children's stderr passes through; their stdout (rank 0's single JSON line) is forwarded.
    Returns the child's exit status (non-zero if any rank failed)."""
    import socket
    import subprocess

    backend = os.environ.get("MGN_DIST_BACKEND", "nccl")
    if backend == "nccl" and not a.dry:
        ndev = torch.cuda.device_count()  # counts devices without initialising HIP on this image
        if ndev < a.gpus:
            print("bench.py: --gpus %d but %d GPU(s) visible (one RCCL rank per GPU; MGN_DIST_BACKEND=gloo "
                  "rehearses several ranks per GPU)" % (a.gpus, ndev), file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % a.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MGN_BENCH_LAUNCHED="%d" % a.gpus)
    print("[bench] starting %d ranks: %s" % (a.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    for line in p.stdout:
        if line.startswith("{"):
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    return p.wait()


def dry_run(a, rank, world):
    """--dry: the process group of the launched ranks (gloo, no device), every rank's (rank, world) agreed
    by an all_gather; rank 0 prints the fields the bench line would carry."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        import socket

        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = torch.tensor([rank, world], dtype=torch.int64)
    allv = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allv, mine)
    ranks = sorted(int(t[0]) for t in allv)
    if ranks != list(range(world)) or any(int(t[1]) != world for t in allv):
        raise RuntimeError("ranks disagree on the world: %s" % [t.tolist() for t in allv])
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry": True, "n_gpus": world, "ranks": ranks,
                          "launched_by": "bench.py" if os.environ.get("MGN_BENCH_LAUNCHED") else "external",
                          "config": {"parallelism": "dp%d" % world}}), file=OUT, flush=True)
    dist.destroy_process_group()


def main():
    a = parse()
    if a.print_workload:
        print(workload_key(a))
        return
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    # the JSON line is the only thing on stdout: everything else written to file descriptor 1 (gloo's
    # "[Gloo] Rank ... connected" lines, library prints) goes to stderr
    global OUT
    sys.stdout.flush()
    OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != a.gpus:
        print("[bench rank %d] --gpus %d under a launcher of %d rank(s): measuring %d" % (rank, a.gpus, world, world),
              file=sys.stderr, flush=True)
        a.gpus = world
    if a.dry:
        dry_run(a, rank, world)
        return
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
    from graphphysics.utils import meshes

    t_start = time.perf_counter()

    def log(msg):  # progress on stderr (the JSON line stays the only stdout line)
        print("[bench rank %d %.1fs] %s" % (rank, time.perf_counter() - t_start, msg), file=sys.stderr, flush=True)

    nat.load()
    mesh = meshes.load_cylinder_mesh()
    step, sim, b, data, lay, workload, datadesc = build_step(a, dev, rank, mesh, world)
    N, E = data.x.shape[0], data.edge_index.shape[1]
    log("step built (N=%d, E=%d, world=%d)" % (N, E, world))
    warm(a, step)
    log("warm-up done (%s)" % ("graph captured" if step.use_graph else "eager"))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    base = {k: getattr(data, k) for k in ("x", "y", "edge_index", "edge_attr")}

    def fresh():
        # a new Batch per step, as the Lightning loop collates: new tensors (topology cache miss)
        for k, v in base.items():
            setattr(data, k, v.clone())

    ctl0 = step.ctl_seconds
    t0 = time.perf_counter()
    for _ in range(a.steps):
        if a.fresh_batch:
            fresh()
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctl_ms = 1000 * (step.ctl_seconds - ctl0) / a.steps  # host gloo re-capture agreement (N > 1, graph mode)
    log("timed steps done: %.3f ms/step" % (1000 * dt / a.steps))
    # sustained rate: the same step replayed for about `sustain` more seconds (reported beside the
    # headline, never as `value`; it also keeps the GPU visibly busy for the driver's sampler)
    sus = None
    if a.sustain > 0 and not a.fresh_batch:
        n_s = max(int(a.sustain / max(dt / a.steps, 1e-4)), a.steps)
        if world > 1:  # every rank replays the same count (collectives inside the step)
            t = torch.tensor([n_s], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            n_s = int(t.item())
        t1 = time.perf_counter()
        for _ in range(n_s):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        ds = time.perf_counter() - t1
        sus = {"steps": n_s, "seconds": round(ds, 3), "value": round(world * n_s / ds, 3), "unit": "steps/s"}
        log("sustained: %d steps in %.2f s" % (n_s, ds))
    prof = profile_classes(a, step) if not a.no_profile else {}
    nparams = sum(p.numel() for p in sim.parameters())
    dp_info = None
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
        # every rank ran the same configuration: world size, parameter count, and (overlapped
        # all-reduce) gradient buckets that covered every parameter exactly once
        covered = step.buckets.covered if (step.overlap and step.buckets is not None) else -1
        if covered >= 0 and covered != nparams:
            raise RuntimeError("gradient buckets covered %d of %d parameters" % (covered, nparams))
        chk = torch.tensor([dist.get_world_size(), nparams, covered, a.batch, a.mp, a.hidden],
                           device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.int64)
        allc = [torch.empty_like(chk) for _ in range(world)]
        dist.all_gather(allc, chk)
        if any(not torch.equal(c, chk) for c in allc):
            raise RuntimeError("ranks disagree on (world, params, covered, batch, mp, hidden): %s"
                               % [c.tolist() for c in allc])
        stats = getattr(sim, "_stats_buf", None)
        dp_info = {"world_size": dist.get_world_size(), "world_size_agreed_by_all_ranks": True,
                   "grad_allreduce_bytes_per_step": 4 * nparams,
                   "stats_allreduce_bytes_per_step": 4 * stats.numel() if stats is not None else None,
                   "grad_buckets_cover_all_params": covered == nparams if covered >= 0 else None,
                   "grad_buckets_per_step": step.buckets.issued if (step.overlap and step.buckets) else None,
                   "recapture_agreement_ms_per_step": round(ctl_ms, 4),
                   "recapture_agreement": "host gloo MAX all-reduce of one int per step (TrainStep._ctl), inside "
                                          "the timed region",
                   "backend": dist.get_backend()}
    last_loss = float(loss.item())

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    kinds, roof = analyse(a, prof, sim, lay, N, E, dt)
    # value: per-GPU training steps (one batch of a.batch graphs each) completed by ALL ranks per second
    # (whole-job aggregate, weak scaling). With N ranks one optimizer step consumes N such batches:
    # the optimizer-step rate and the graph rate are reported separately.
    value = world * a.steps / dt
    gpb = a.batch if a.workload == "cylinder" else 1
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "steps/s", "n_gpus": world, "steps": a.steps,
        "value_definition": "per-GPU training steps (batch of %d graphs) of all %d rank(s) per second; "
                            "= optimizer_steps_per_s x n_gpus" % (gpb, world),
        "optimizer_steps_per_s": round(a.steps / dt, 3), "graphs_per_s": round(value * gpb, 2),
        "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": a.dtype,
        "data": "synthetic: %s, random-init weights (seed 0)" % datadesc,
        "execution": ("eager, a new batch (fresh x / y / edge_index / edge_attr tensors, topology rebuilt) "
                      "every step" if a.fresh_batch else "eager" if not step.use_graph else
                      ("hipGraph replay of the whole data-parallel step: statistics + mask-count all-reduce, "
                       "forward+loss+backward with the bucketed gradient all-reduce overlapped on a communication "
                       "stream, AdamW"
                       if step.overlap else
                       "hipGraph replay of forward+loss+backward; eager statistics/gradient all-reduce + AdamW")
                      if step.dp else "hipGraph replay of the whole step"),
        "config": {"workload": workload, "nodes_per_gpu": N, "edges_per_gpu": E,
                   "global_batch": (a.batch if a.workload == "cylinder" else 1) * world,
                   "parallelism": "dp%d" % world,
                   "graphs_per_sec": round(value * gpb, 2)},
        "roofline": roof, "kernels": kinds, "kernels_schedule": PROFILE_SCHEDULE, "last_loss": last_loss,
    }
    if dp_info is not None:
        out["data_parallel"] = dp_info
    if sus is not None:
        out["sustained"] = sus

    if world == 1 and roof is not None:
        roof["scatter_standalone"] = scatter_standalone(a, data, dev)
    if not a.no_mse and a.workload == "cylinder":
        out["one_step_mse"] = one_step_mse(sim, mesh, dev, a)
    if world == 1 and a.cpu_steps > 0:
        out["cpu_baseline"] = cpu_baseline(a, b, lay)
        if out["cpu_baseline"]:
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
    if world == 1 and not a.no_secondary and a.workload == "cylinder":
        # BASELINE.md Config B in the reference's fp32 and Config A (training_config/cylinder.json
        # as written: MP=5, h=32, fp32, one graph) with its CPU baseline, same invocation
        del step, sim
        torch.cuda.empty_cache()
        sec = {}
        if not (a.dtype == "fp32" and a.mp == 15 and a.hidden == 128 and a.batch == 8):
            sec["cfgB_fp32"] = secondary(a, dev, mesh, "Config B in fp32 (the reference's dtype)", dtype="fp32",
                                         mp=15, hidden=128, batch=8)
        sec["cfgA"] = secondary(a, dev, mesh, "Config A: training_config/cylinder.json (MP=5, h=32, fp32, B=1)",
                                cpu_steps=(20 if a.cpu_steps > 0 else 0), dtype="fp32", mp=5, hidden=32, batch=1)
        # BASELINE config 2 at training_config/plate.json's sizes (MP=10, h=64; the reference file
        # selects its transformer processor, out of scope: this is the MGN processor at those sizes)
        sec["cfgC_plate"] = secondary(a, dev, mesh, "Config C: DeformingPlate MGN at plate.json's sizes (MP=10, h=64, "
                                      "bf16), world edges + relative-position features, 1 graph",
                                      dtype="bf16", mp=10, hidden=64, batch=1, workload="plate")
        # BASELINE config 4 per GPU (Cfg E): the reference's aneurysm mesh, k-hop 2 built on device
        # (N=22,535, E=1,395,256), MP=15, h=128, bf16 — the largest single-GPU workload
        sec["cfgE_aneurysm"] = secondary(a, dev, mesh, "Config E per GPU: 3D-CoarseAneurysm, k-hop 2 (1 graph, "
                                         "N=22,535, E=1,395,256), MP=15, h=128, bf16", dtype="bf16", mp=15,
                                         hidden=128, batch=1, workload="aneurysm")
        out["secondary"] = sec
    print(json.dumps(out), file=OUT, flush=True)
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


def replay_lookup(workload):
    """Per-class device time of the replayed step from the newest committed profiles/*_traffic.json
    recorded on the same kernel sources (sha256 stamp) and workload (tools/pmc_traffic.py `replay`)."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import sources_sha

    sha = sources_sha()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        d = json.load(open(f))
        if d.get("sources_sha") == sha and d.get("workload") == workload and d.get("replay"):
            return {"source": os.path.relpath(f, ROOT), "replay": d["replay"]}
    return {}


def pmc_lookup(kernel_class, workload):
    """PMC figures of `kernel_class` from the newest committed profiles/*_traffic.json measured on the
    same kernel sources (sha256 stamp) AND the same workload, averaged over that class's kernel
    instances weighted by their launches (the class time bench.py reports averages the same launches).
    Only records whose PMC passes ran on one stream (tools/profile_round.sh: MGN_CONC_WGRAD=0), the
    schedule of bench.py's per-class timing."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import sources_sha

    sha = sources_sha()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), reverse=True):
        d = json.load(open(f))
        if d.get("sources_sha") != sha or d.get("workload") != workload:
            continue
        if not d.get("schedule", "").startswith("one stream"):
            continue  # a record of the concurrent schedule describes other launches than avg_launch_us times
        inst = [v for v in d.get("kernels", {}).values() if v.get("class") == kernel_class]
        out = {"source": os.path.relpath(f, ROOT), "instances": [v["kernel"][:80] + " grid=" + v["grid"] for v in inst],
               "schedule": d.get("schedule", "default (MGN_CONC_WGRAD=auto)")}
        for field in ("hbm_bytes", "mfma_util", "trace_us", "grbm_us_at_2400MHz", "implied_clock_mhz"):
            vals = [(v[field], v.get("launches", 1)) for v in inst if field in v]
            if vals:
                out[field] = round(sum(x * w for x, w in vals) / sum(w for _, w in vals), 4 if field == "mfma_util" else 0
                                   if field == "hbm_bytes" else 2)
        return out
    return {"source": "no PMC pass on these kernel sources and workload (run tools/profile_round.sh)"}


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


def cpu_baseline(a, b, lay, warmup=3):
    """The reference algorithm on the host (oracle = op-for-op restatement of the reference's
    PyTorch CPU path, pinned to golden vectors), same workload, fp32, all cores: `warmup` untimed
    steps, then a.cpu_steps timed ones, median."""
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

    for _ in range(warmup):
        step()
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
            "sample": "%d timed + %d warm-up full training steps of the same workload (MP=%d, h=%d, N=%d, E=%d), "
                      "torch %s fp32, median" % (a.cpu_steps, warmup, a.mp, a.hidden, b["x"].shape[0],
                                                 b["edge_index"].shape[1], torch.__version__),
            "cpu": model, "host": platform.node()}


if __name__ == "__main__":
    main()
