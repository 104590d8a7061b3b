"""Graph-construction oracle (oracle/graph_oracle.py) pinned to the reference (CPU, no GPU).

Pins: the reference test's edge counts (CylinderFlow mock mesh: 11070 edges, 32638 at k-hop 2 —
reference tests/graphphysics/dataset/test_xdmfdataset.py:173-175,228-230) and golden vectors from
the reference's own compute_k_hop_edge_index (tests/golden/make_graph_golden.py). Bit-exact.
"""
import os

import numpy as np
import torch

from oracle import graph_oracle as GO

G = os.path.join(os.path.dirname(__file__), "golden")


def _z(name):
    z = np.load(os.path.join(G, name))
    return {k: z[k] for k in z.files}


def _cyl_edges():
    m = _z("cylinder_mesh.npz")
    n = m["pos"].shape[0]
    return GO.face_to_edge(torch.from_numpy(m["triangles"].astype(np.int64)).t().contiguous(), n), n


def test_cylinder_face_to_edge_count_and_order():
    ei, n = _cyl_edges()
    assert ei.shape == (2, 11070)
    key = ei[0] * n + ei[1]
    assert bool((key[1:] > key[:-1]).all())  # coalesced: strictly increasing (row, col)
    # undirected: the reversed list is the same set
    assert torch.equal(GO.to_undirected(ei.flip(0), n), ei)


def test_cylinder_khop_matches_reference_golden():
    ei, n = _cyl_edges()
    g = _z("graph_golden.npz")
    for k in (2, 3):
        kh = GO.k_hop_edge_index(ei, k, n)
        np.testing.assert_array_equal(kh.numpy(), g[f"cyl_khop{k}"].astype(np.int64))
    assert g["cyl_khop2"].shape[1] == 32638


def test_aneurysm_tetra_edges_and_khop_digest():
    a, g = _z("aneurysm_mesh.npz"), _z("graph_golden.npz")
    n = a["pos"].shape[0]
    ei = GO.face_to_edge(torch.from_numpy(a["tetra"].astype(np.int64)).t().contiguous(), n)
    assert ei.shape[1] == int(g["an_khop1_count"]) == 291144
    assert GO.pattern_digest(ei) == str(g["an_khop1_sha"])
    kh = GO.k_hop_edge_index(ei, 2, n)
    assert kh.shape[1] == int(g["an_khop2_count"]) == 1395256
    assert GO.pattern_digest(kh) == str(g["an_khop2_sha"])
    assert int(torch.bincount(kh[1], minlength=n).max()) == int(g["an_khop2_max_indeg"]) == 103


def test_world_edges_semantics_small():
    # 4 points on a line, spacing 0.02: radius 0.03 links neighbours only; only OBSTACLE–NORMAL kept
    pos = torch.tensor([[0.0, 0, 0], [0.02, 0, 0], [0.04, 0, 0], [0.06, 0, 0]])
    nt = torch.tensor([1.0, 0.0, 0.0, 1.0])
    mesh = torch.zeros((2, 0), dtype=torch.long)
    ei = GO.world_edges(pos, nt, mesh, 0.03)
    assert ei.tolist() == [[0, 1, 2, 3], [1, 0, 3, 2]]
