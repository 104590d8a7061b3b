"""Round 5, VERDICT r04 item 3 (bytes-first A/B, measured): what the edge MLP's backward saves cost the
block forward. The same 15-block bf16 h=128 EncodeProcessDecode forward on a bench workload twice —
training mode (R8 saves of every hidden layer's input, ReLU mask words, z, rden) and inference mode
(mgn_block_forward with act = NULL: z and rden only, the aggregation's inputs) — per-class kernel times
from libmgn's HIP-event profiler. Run it under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE for the bytes of
chain16_fwd_kernel<true,...> (training) vs <false,...> (inference).

    python tools/dev/r05_saves.py cylinder|aneurysm [iters]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "graph-physics_amd")]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "cylinder"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import __graft_entry__ as ge

    ge._paths()
    import bench
    from graphphysics import _native as nat
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    nat.load()
    dev = torch.device("cuda", 0)
    a = argparse.Namespace(workload=wl, batch=8, mp=15, hidden=128, dtype="bf16")
    _, data, lay, _, _ = bench.make_workload(a, dev, 0, meshes.load_cylinder_mesh())
    N, E = data.x.shape[0], data.edge_index.shape[1]
    torch.manual_seed(0)
    model = EncodeProcessDecode(15, lay["node_in"], lay["edge_in"], lay["out"], 128, compute_dtype=torch.bfloat16).to(dev)
    g = Data(x=torch.randn(N, lay["node_in"], device=dev), edge_index=data.edge_index,
             edge_attr=torch.randn(E, lay["edge_in"], device=dev))
    res = {"workload": wl, "nodes": N, "edges": E}
    for mode in ("train", "infer"):
        for _ in range(3):
            if mode == "train":
                model(g)
            else:
                with torch.no_grad():
                    model(g)
        torch.cuda.synchronize()
        nat.profile_enable(True)
        for _ in range(iters):
            if mode == "train":
                model(g)
            else:
                with torch.no_grad():
                    model(g)
        torch.cuda.synchronize()
        prof = nat.profile_collect()
        nat.profile_enable(False)
        res[mode] = {k: {"avg_us": round(1000 * ms / cnt, 2), "launches_per_fwd": cnt / iters}
                     for k, (ms, cnt) in prof.items() if cnt}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
