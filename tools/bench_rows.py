"""Measurements for the SURVEY.md §8(f) rows beside the headline training step (bench.py):

  rollout      autoregressive validation rollout (graphphysics.training.rollout.Rollout, hipGraph
               replay, inference block kernels) on the Cfg B batch (8 CylinderFlow graphs, MP=15,
               h=128, bf16): rollout steps/s, per-kernel HIP-event times of the inference edge kernel
               and its HBM roofline; CPU baseline = the oracle's eval forward (reference ops) on the
               same batch.
  graph_build  on-device construction of the Cfg E graph (3D aneurysm mock mesh, N=22,535, 115,275
               tetrahedra): FaceToEdge (291,144 edges), k-hop 2 (1,395,256 edges), Cartesian+Distance
               features; CPU baseline = the oracle (PyG-semantics restatement / the reference's
               torch.sparse k-hop) on the same mesh.
  world_edges  radius-0.03 OBSTACLE–NORMAL pairs on a DeformingPlate-shaped synthetic 3D cloud
               (20,000 nodes) + to_undirected; CPU baseline = scipy cKDTree (the reference's call).

    python tools/bench_rows.py [--steps 50] > gpurun_out/rows.json
Prints ONE JSON object. GPU times: wall clock around synchronised calls (graph construction
returns counts to the host, as the reference's does) or HIP events (kernel classes).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]
HBM_PEAK = 8000.0
MFMA_PEAK_BF16 = 2500.0  # TFLOP/s, dense bf16 (MI355X_MICROARCH.md)


def timed(fn, reps, sync=True):
    ts = []
    for _ in range(reps):
        if sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), out


def rollout_row(a, dev):
    from oracle import mgn_oracle as O
    from graphphysics import _native as nat
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.rollout import Rollout
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    mesh = meshes.load_cylinder_mesh()
    frames = []
    for t in range(5):
        b = meshes.cylinder_batch(8, t=t, jitter=0.01, mesh=mesh)
        frames.append(Data(**{k: torch.from_numpy(b[k]).to(dev) for k in ("x", "y", "edge_index", "edge_attr")}))
    frames = [Data(x=f.x, y=f.y, edge_index=frames[0].edge_index, edge_attr=frames[0].edge_attr) for f in frames]
    torch.manual_seed(0)
    model = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16)
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, model, dev)
    with torch.no_grad():
        sim(frames[0])  # normaliser statistics
    sim.eval()
    ro = Rollout(sim, 2, graph=True)
    seq = [frames[i % len(frames)] for i in range(a.steps)]
    ro.rollout(seq[:5])  # warm-up + graph record
    ro.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ro.rollout(seq)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # per-kernel times of the inference forward (eager, same kernels as the replay)
    nat.profile_enable(True)
    for f in seq[:10]:
        ro._eager(f)
    torch.cuda.synchronize()
    prof = nat.profile_collect()
    nat.profile_enable(False)
    n, e, h = frames[0].x.shape[0], frames[0].edge_index.shape[1], 128
    kern = {k: {"avg_us": round(1000 * ms / c, 2), "launches": c} for k, (ms, c) in prof.items() if c}
    # MLP kernels on the MFMA roof. The inference edge kernel runs 8h² FLOPs per edge
    # (layer 0's e block + three h x h Linears; the x blocks are the node projections); one rollout
    # step is one forward F_fwd = MP (12h²E + 10h²N) + encoders + decoder
    fe = kern.get("fwd_edge")
    roof = None
    f_fwd = 15 * (12 * h * h * e + 10 * h * h * n) + 2 * (3 * h + 3 * h * h) * e + 2 * (11 * h + 3 * h * h) * n \
        + 2 * (3 * h * h + 2 * h) * n
    if fe:
        fl = 8 * h * h * e
        tf = fl / (fe["avg_us"] * 1e-6) / 1e12
        roof = {"kernel": "fwd_edge (inference)", "bound": "mfma", "achieved": round(tf, 2), "peak": MFMA_PEAK_BF16,
                "unit": "TFLOP/s", "frac": round(tf / MFMA_PEAK_BF16, 4), "flops_per_launch": fl,
                "avg_launch_us": fe["avg_us"],
                # the same kernel's compulsory bytes (e in, e' / z out bf16, rden, fp32 P_i/P_j gathers)
                "hbm_gbs": round(e * (3 * 2 * h + 4 + 2 * 4 * h) / (fe["avg_us"] * 1e-6) / 1e9, 1)}
    # CPU baseline: the oracle's eval forward on the same batch (reference ops, fp32)
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    ref = O.OracleEPD(15, 11, 3, 2, 128)
    ref.load_state_dict({k: v.detach().float().cpu() for k, v in sim.model.state_dict().items()})
    osim = O.OracleSimulator(ref, 11, 3, 2)
    f0 = frames[0]
    x, y, ei, ea = (f0.x.cpu(), f0.y.cpu(), f0.edge_index.cpu(), f0.edge_attr.cpu())
    with torch.no_grad():
        osim.forward(x, y, ei, ea, training=True)
        t_cpu, _ = timed(lambda: osim.forward(x, y, ei, ea, training=False), a.cpu_forwards, sync=False)
    step_tf = f_fwd * a.steps / dt / 1e12
    return {"value": round(a.steps / dt, 2), "unit": "rollout steps/s", "ms_per_step": round(1000 * dt / a.steps, 3),
            "step_mfma": {"flops_per_step": f_fwd, "tflops_per_s": round(step_tf, 2),
                          "frac": round(step_tf / MFMA_PEAK_BF16, 4), "note": "F_fwd (SURVEY §8d) / measured ms_per_step"},
            "steps": a.steps, "config": {"workload": "Cfg B rollout: 8 CylinderFlow graphs, MP=15, h=128, bf16",
                                         "nodes": n, "edges": e},
            "execution": "hipGraph replay per step (inference block kernels)", "roofline": roof, "kernels": kern,
            "cpu_baseline": {"value": round(1.0 / t_cpu, 4), "unit": "rollout steps/s", "cores": cores,
                             "kind": "port", "sample": "%d timed eval forwards (median) of the same batch "
                                                       "after one warm-up (oracle, fp32)" % a.cpu_forwards}}


def graph_row(dev):
    from oracle import graph_oracle as GO
    from graphphysics.utils import graph_build as G

    z = np.load(os.path.join(ROOT, "tests", "golden", "aneurysm_mesh.npz"))
    pos, tet = torch.from_numpy(z["pos"]), torch.from_numpy(z["tetra"].astype(np.int64)).t().contiguous()
    n = pos.shape[0]
    pd, td = pos.to(dev), tet.to(dev)
    G.face_to_edge(td, n)  # warm-up
    t_f2e, ei = timed(lambda: G.face_to_edge(td, n), 5)
    G.k_hop_edge_index(ei, 2, n)
    t_kh, kh = timed(lambda: G.k_hop_edge_index(ei, 2, n), 5)
    t_ef, _ = timed(lambda: G.edge_features(pd, kh), 5)
    e1, e2 = ei.shape[1], kh.shape[1]
    cores = torch.get_num_threads()
    c_f2e, cei = timed(lambda: GO.face_to_edge(tet, n), 1, sync=False)
    c_kh, ckh = timed(lambda: GO.k_hop_edge_index(cei, 2, n), 1, sync=False)
    c_ef, _ = timed(lambda: GO.edge_features(pos, ckh), 1, sync=False)
    assert GO.pattern_digest(kh.cpu()) == GO.pattern_digest(ckh)
    # edge-feature kernel bytes: 2 int64 indices + 2 gathered fp32 3-vectors + 4 fp32 out per edge
    efb = e2 * (16 + 24 + 16)
    return {"workload": "Cfg E graph: 3D aneurysm mock mesh, N=%d, %d tetrahedra" % (n, tet.shape[1]),
            "face_to_edge": {"edges": e1, "gpu_ms": round(1e3 * t_f2e, 3), "cpu_ms": round(1e3 * c_f2e, 1),
                             "speedup": round(c_f2e / t_f2e, 1)},
            "k_hop_2": {"edges": e2, "gpu_ms": round(1e3 * t_kh, 3), "cpu_ms": round(1e3 * c_kh, 1),
                        "speedup": round(c_kh / t_kh, 1), "gpu_edges_per_s": round(e2 / t_kh, 1)},
            "edge_features": {"edges": e2, "gpu_ms": round(1e3 * t_ef, 3), "cpu_ms": round(1e3 * c_ef, 1),
                              "speedup": round(c_ef / t_ef, 1),
                              "roofline": {"bound": "hbm", "achieved": round(efb / t_ef / 1e9, 1), "peak": HBM_PEAK,
                                           "unit": "GB/s", "frac": round(efb / t_ef / 1e9 / HBM_PEAK, 4),
                                           "note": "wall clock incl. the range check's host read-back"}},
            "cpu_baseline": {"kind": "port", "cores": cores,
                             "sample": "oracle (PyG-semantics FaceToEdge, reference torch.sparse k-hop), 1 run each"},
            "parity": "k-hop edge list sha256 identical to the CPU oracle's"}


def world_row(dev):
    from oracle import graph_oracle as GO
    from graphphysics.utils import graph_build as G

    gen = torch.Generator().manual_seed(3)
    n = 20000
    pos = torch.rand(n, 3, generator=gen) * torch.tensor([1.0, 0.3, 0.3])
    nt = (torch.rand(n, generator=gen) < 0.1).float()
    mesh = torch.zeros((2, 0), dtype=torch.long)
    pd, nd, md = pos.to(dev), nt.to(dev), mesh.to(dev)

    def gpu():
        added = G.radius_pairs(pd, 0.03, node_type=nd)
        return G.to_undirected(torch.cat([added, md], 1), n)

    gpu()
    t_g, got = timed(gpu, 5)
    t_c, ref = timed(lambda: GO.world_edges(pos, nt, mesh, 0.03), 1, sync=False)
    assert torch.equal(got.cpu(), ref)
    return {"workload": "synthetic DeformingPlate-shaped cloud, %d nodes, r=0.03, 10%% OBSTACLE" % n,
            "edges": int(ref.shape[1]), "gpu_ms": round(1e3 * t_g, 3), "cpu_ms": round(1e3 * t_c, 1),
            "speedup": round(t_c / t_g, 1), "cpu_baseline": {"kind": "reference-dependency",
                                                             "sample": "scipy cKDTree.query_pairs + mask + to_undirected"},
            "parity": "identical edge list"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--cpu-forwards", type=int, default=10, help="timed CPU (oracle) eval forwards")
    a = ap.parse_args()
    import __graft_entry__ as ge

    ge.build()
    dev = torch.device("cuda:0")
    out = {"rows": "SURVEY.md §8(f) 1, 3, 4"}
    out["rollout"] = rollout_row(a, dev)
    out["graph_build"] = graph_row(dev)
    out["world_edges"] = world_row(dev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
