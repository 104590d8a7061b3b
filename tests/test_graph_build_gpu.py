"""On-device graph construction (libmgn mgn_build.hip) vs the oracle and the reference's golden
vectors.

Tolerances: every index set (FaceToEdge, to_undirected/coalesce, k-hop, radius pairs, world
edges) bit-exact — same edges in the same (row, col)-sorted order; edge features (fp32
subtraction exact, the norm within 2 ulp of torch.norm: rtol 2.5e-7, atol 1e-12).
"""
import os

import numpy as np
import pytest
import torch

from oracle import graph_oracle as GO

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _built():
    import __graft_entry__ as ge

    ge.build()
    assert torch.cuda.is_available(), "GPU tests need a HIP device"


def _z(name):
    z = np.load(os.path.join(G, name))
    return {k: z[k] for k in z.files}


def _gb():
    from graphphysics.utils import graph_build

    return graph_build


def test_face_to_edge_cylinder_and_aneurysm():
    gb = _gb()
    m = _z("cylinder_mesh.npz")
    n = m["pos"].shape[0]
    face = torch.from_numpy(m["triangles"].astype(np.int64)).t().contiguous()
    ei = gb.face_to_edge(face.to(DEV), n).cpu()
    assert torch.equal(ei, GO.face_to_edge(face, n)) and ei.shape == (2, 11070)
    a, g = _z("aneurysm_mesh.npz"), _z("graph_golden.npz")
    tet = torch.from_numpy(a["tetra"].astype(np.int64)).t().contiguous()
    ea = gb.face_to_edge(tet.to(DEV), a["pos"].shape[0]).cpu()
    assert ea.shape[1] == 291144 and GO.pattern_digest(ea) == str(g["an_khop1_sha"])


def test_khop_matches_reference_golden():
    gb = _gb()
    m, g = _z("cylinder_mesh.npz"), _z("graph_golden.npz")
    n = m["pos"].shape[0]
    face = torch.from_numpy(m["triangles"].astype(np.int64)).t().contiguous()
    ei = gb.face_to_edge(face.to(DEV), n)
    for k in (2, 3):
        np.testing.assert_array_equal(gb.k_hop_edge_index(ei, k, n).cpu().numpy(),
                                      g[f"cyl_khop{k}"].astype(np.int64))
    a = _z("aneurysm_mesh.npz")
    na = a["pos"].shape[0]
    ea = gb.face_to_edge(torch.from_numpy(a["tetra"].astype(np.int64)).t().contiguous().to(DEV), na)
    kh = gb.k_hop_edge_index(ea, 2, na).cpu()
    assert kh.shape[1] == 1395256 and GO.pattern_digest(kh) == str(g["an_khop2_sha"])


@pytest.mark.parametrize("n,e,seed", [(50, 300, 0), (1000, 20000, 1), (7, 0, 2), (1, 5, 3)])
def test_coalesce_khop_random_multigraph(n, e, seed):
    """Unsorted input with duplicates and self loops (the reference coalesces its input first)."""
    gb = _gb()
    gen = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, e), generator=gen)
    d = ei.to(DEV)
    assert torch.equal(gb.to_undirected(d, n).cpu(), GO.to_undirected(ei, n))
    assert torch.equal(gb.coalesce(d, n).cpu(), GO.coalesce_pattern(ei[0], ei[1], n))
    nosl = GO.coalesce_pattern(ei[0], ei[1], n)
    nosl = nosl[:, nosl[0] != nosl[1]]
    assert torch.equal(gb.coalesce(d, n, drop_self_loops=True).cpu(), nosl)
    for k in (2, 3):
        assert torch.equal(gb.k_hop_edge_index(d, k, n).cpu(), GO.k_hop_edge_index(ei, k, n))


def test_out_of_range_raises_index_error():
    gb = _gb()
    ei = torch.tensor([[0, 1, 5], [1, 2, 0]], device=DEV)
    with pytest.raises(IndexError):
        gb.to_undirected(ei, 5)
    with pytest.raises(IndexError):
        gb.k_hop_edge_index(ei, 2, 5)
    with pytest.raises(IndexError):
        gb.face_to_edge(torch.tensor([[0], [1], [9]], device=DEV), 5)
    with pytest.raises(IndexError):
        gb.edge_features(torch.zeros(5, 2, device=DEV), ei)


def test_refuses_cpu_tensors():
    gb = _gb()
    with pytest.raises(RuntimeError, match="HIP device"):
        gb.to_undirected(torch.zeros((2, 1), dtype=torch.long), 2)


def test_edge_features_vs_oracle():
    gb = _gb()
    gen = torch.Generator().manual_seed(5)
    for dim in (2, 3):
        pos = torch.randn(500, dim, generator=gen)
        ei = torch.randint(0, 500, (2, 4000), generator=gen)
        got = gb.edge_features(pos.to(DEV), ei.to(DEV)).cpu()
        ref = GO.edge_features(pos, ei)
        assert torch.equal(got[:, :dim], ref[:, :dim])
        torch.testing.assert_close(got[:, dim], ref[:, dim], rtol=2.5e-7, atol=1e-12)


@pytest.mark.parametrize("dim,n,r", [(3, 3000, 0.08), (2, 2000, 0.05), (3, 1, 0.1), (3, 500, 10.0)])
def test_radius_pairs_vs_ckdtree(dim, n, r):
    gb = _gb()
    gen = torch.Generator().manual_seed(dim * 100 + n)
    pos = torch.rand(n, dim, generator=gen)
    got = gb.radius_pairs(pos.to(DEV), r).cpu()
    ref = GO.radius_pairs(pos, r)
    key = lambda p: torch.sort(p[0] * n + p[1]).values  # noqa: E731  (pair order unspecified)
    assert got.shape == ref.shape and torch.equal(key(got), key(ref))
    assert bool((got[0] < got[1]).all()) if got.numel() else True


def test_world_edges_vs_oracle():
    """add_world_edges (reference preprocessing.py:92-140): DeformingPlate-shaped tet mesh + obstacle."""
    from graphphysics.dataset.preprocessing import add_world_edges
    from graphphysics.utils.data import Data

    gb = _gb()
    gen = torch.Generator().manual_seed(11)
    n = 1200
    pos = torch.rand(n, 3, generator=gen) * 0.3
    nt = (torch.rand(n, generator=gen) < 0.2).float()  # 1 = OBSTACLE, 0 = NORMAL
    nt[:40] = 3.0  # HANDLE nodes never get world edges
    cells = torch.randint(0, n, (4, 2000), generator=gen)
    mesh = GO.face_to_edge(cells, n)
    x = torch.cat([pos, torch.randn(n, 2, generator=gen), nt[:, None]], 1)
    ref = GO.world_edges(pos, nt, mesh, 0.03)
    g = Data(x=x.to(DEV), edge_index=gb.face_to_edge(cells.to(DEV), n))
    g = add_world_edges(g, 0, 3, 5, radius=0.03)
    assert torch.equal(g.edge_index.cpu(), ref)
    assert ref.shape[1] > mesh.shape[1]  # some world edges were added


def test_k_hop_graph_and_preprocessing_pipeline():
    """compute_k_hop_graph with edge features + build_preprocessing(FaceToEdge, Cartesian, Distance)."""
    from graphphysics.dataset.preprocessing import build_preprocessing
    from graphphysics.utils.data import Data
    from graphphysics.utils.torch_graph import compute_k_hop_graph

    m = _z("cylinder_mesh.npz")
    n = m["pos"].shape[0]
    face = torch.from_numpy(m["triangles"].astype(np.int64)).t().contiguous()
    pos = torch.from_numpy(m["pos"].astype(np.float32))
    x = torch.randn(n, 3)
    g = build_preprocessing()(Data(x=x.to(DEV), pos=pos.to(DEV), face=face.to(DEV)))
    ei = GO.face_to_edge(face, n)
    assert torch.equal(g.edge_index.cpu(), ei)
    ref = GO.edge_features(pos, ei)
    torch.testing.assert_close(g.edge_attr.cpu(), ref, rtol=2.5e-7, atol=1e-12)
    kg = compute_k_hop_graph(g, 2, add_edge_features_to_khop=True, world_pos_index_start=None,
                             world_pos_index_end=None)
    kei = GO.k_hop_edge_index(ei, 2, n)
    assert torch.equal(kg.edge_index.cpu(), kei)
    torch.testing.assert_close(kg.edge_attr.cpu(), GO.edge_features(pos, kei), rtol=2.5e-7, atol=1e-12)
    # default world-pos block (x[:, 0:3]) appended (torch_graph.py:101-110): 2D Cartesian + Distance
    # (3 columns) then 3D relative world pos + norm (4 columns)
    kg7 = compute_k_hop_graph(g, 2, add_edge_features_to_khop=True)
    assert kg7.edge_attr.shape == (kei.shape[1], 7)
    torch.testing.assert_close(kg7.edge_attr[:, 3:].cpu(), GO.edge_features(x, kei), rtol=2.5e-7, atol=1e-12)
