"""Golden vectors for on-device graph construction, produced by the
REFERENCE's own compute_k_hop_edge_index (graphphysics/utils/torch_graph.py:16-53 — pure
torch.sparse code) imported from /root/reference with import-only placeholders for meshio and the
PyG transforms/utils it names but this path never calls (tests/golden/_stubs). Run in the build
container only:

    PYTHONPATH=tests/golden/_stubs:/root/reference python tests/golden/make_graph_golden.py

Inputs: the CylinderFlow mock mesh (tests/golden/cylinder_mesh.npz, decoded from the reference's
tests/mock_vtu/cylinder_0.vtu) and the 3D aneurysm mock mesh (reference
tests/mock_vtu_aneurysm/aneurysm_0.vtu, decoded here and committed as
tests/golden/aneurysm_mesh.npz: points + tetrahedra). Their 1-hop edges come from the oracle's
FaceToEdge restatement (pinned by the reference test's count 11070). Writes
tests/golden/graph_golden.npz: full k-hop lists for the cylinder (k = 2, 3), counts + sha256 of
the aneurysm k = 2 list (1.4M edges).
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
assert os.path.isdir(REF), "make_graph_golden.py runs only where the reference is mounted"

from graphphysics.utils.torch_graph import compute_k_hop_edge_index  # noqa: E402  (reference code)

sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from vtu import read_vtu  # noqa: E402

from oracle import graph_oracle as GO  # noqa: E402

torch.set_num_threads(8)


def aneurysm_mesh():
    path = os.path.join(HERE, "aneurysm_mesh.npz")
    if not os.path.exists(path):
        a = read_vtu(os.path.join(REF, "tests", "mock_vtu_aneurysm", "aneurysm_0.vtu"))
        assert (a["types"] == 10).all() and (np.diff(a["offsets"]) == 4).all()  # VTK_TETRA only
        np.savez_compressed(path, pos=a["Points"].astype(np.float32),
                            tetra=a["connectivity"].reshape(-1, 4).astype(np.int32))
    z = np.load(path)
    return z["pos"], z["tetra"]


def main():
    out = {}
    m = np.load(os.path.join(HERE, "cylinder_mesh.npz"))
    n = m["pos"].shape[0]
    ei = GO.face_to_edge(torch.from_numpy(m["triangles"].astype(np.int64)).t().contiguous(), n)
    assert ei.shape[1] == 11070
    for k in (2, 3):
        kh = compute_k_hop_edge_index(ei, k, n)
        out[f"cyl_khop{k}"] = kh.numpy().astype(np.int32)
        print("cylinder k-hop", k, kh.shape)
    assert out["cyl_khop2"].shape[1] == 32638  # reference tests/graphphysics/dataset/test_xdmfdataset.py:228-230
    pos, tet = aneurysm_mesh()
    na = pos.shape[0]
    eia = GO.face_to_edge(torch.from_numpy(tet.astype(np.int64)).t().contiguous(), na)
    out["an_khop1_count"] = np.array(eia.shape[1])
    out["an_khop1_sha"] = np.array(GO.pattern_digest(eia))
    kh = compute_k_hop_edge_index(eia, 2, na)
    out["an_khop2_count"] = np.array(kh.shape[1])
    out["an_khop2_sha"] = np.array(GO.pattern_digest(kh))
    out["an_khop2_max_indeg"] = np.array(int(torch.bincount(kh[1], minlength=na).max()))
    print("aneurysm", eia.shape, kh.shape, out["an_khop2_max_indeg"])
    np.savez_compressed(os.path.join(HERE, "graph_golden.npz"), **out)


if __name__ == "__main__":
    main()
