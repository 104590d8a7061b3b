"""Host-side mesh → graph construction (numpy) for CylinderFlow-shaped inputs.

Mirrors the reference's preprocessing for the inputs the MGN kernels consume:
  * FaceToEdge + to_undirected (coalesced ⇒ edges sorted by (row, col), duplicates removed):
    reference graphphysics/dataset/preprocessing.py:16-23,410 (torch-geometric 2.6.1 transforms).
    Pinned counts: CylinderFlow mock mesh N=1923 → E=11070
    (reference tests/graphphysics/dataset/test_xdmfdataset.py:173-175).
  * tetrahedra → 4 faces → edges: reference graphphysics/utils/torch_graph.py:171-186.
  * edge features Cartesian(norm=False) ‖ Distance(norm=False): preprocessing.py:429-431.
    Sign convention chosen here: pos[row] − pos[col] (PyG 2.6.1 sign unpinned offline; the
    kernels consume edge_attr as given, so parity does not depend on it).
  * block-diagonal batching (PyG Batch): node offsets added per graph, edges stay sorted.
On-device construction is SURVEY.md §8(f) row 1 ("next").
"""
import os

import numpy as np

NORMAL, INFLOW, OUTFLOW, WALL_BOUNDARY = 0, 4, 5, 6


def coalesce_undirected(pairs, n):
    pairs = np.asarray(pairs, dtype=np.int64)
    both = np.concatenate([pairs, pairs[:, ::-1]], 0)
    key = np.unique(both[:, 0] * n + both[:, 1])
    return np.stack([key // n, key % n], 0)


def triangles_to_edge_index(tri, n):
    t = np.asarray(tri, dtype=np.int64)
    pairs = np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [0, 2]]], 0)
    return coalesce_undirected(pairs, n)


def tetra_to_edge_index(tet, n):
    t = np.asarray(tet, dtype=np.int64)
    faces = np.concatenate([t[:, [0, 1, 2]], t[:, [0, 1, 3]], t[:, [0, 2, 3]], t[:, [1, 2, 3]]], 0)
    return triangles_to_edge_index(faces, n)


def khop_edge_index(edge_index, n, hops):
    """k-hop augmented adjacency without self loops (reference utils/torch_graph.py:16-53),
    returned coalesced (sorted by (row, col))."""
    import scipy.sparse as sp

    a = sp.csr_matrix((np.ones(edge_index.shape[1]), (edge_index[0], edge_index[1])), shape=(n, n))
    ak = a.copy()
    for _ in range(hops - 1):
        ak = ak + ak @ a
        ak.setdiag(0)
        ak.eliminate_zeros()
    ak = ak.tocoo()
    key = np.unique(ak.row.astype(np.int64) * n + ak.col)
    return np.stack([key // n, key % n], 0)


def edge_features(pos, edge_index):
    d = pos[edge_index[0]] - pos[edge_index[1]]
    return np.concatenate([d, np.linalg.norm(d, axis=1, keepdims=True)], 1).astype(np.float32)


def cylinder_node_types(pos, vel0):
    """Synthetic CylinderFlow node types: INFLOW at x=0, OUTFLOW at x=1.6,
    WALL_BOUNDARY where |v|=0 elsewhere, NORMAL otherwise."""
    nt = np.full(pos.shape[0], NORMAL, np.int64)
    inflow = pos[:, 0] == 0.0
    outflow = pos[:, 0] >= 1.6 - 1e-6
    wall = (np.linalg.norm(vel0, axis=1) == 0) & ~inflow & ~outflow
    nt[inflow], nt[outflow], nt[wall] = INFLOW, OUTFLOW, WALL_BOUNDARY
    return nt


def repo_root():
    return os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))


def load_cylinder_mesh(path=None):
    """The reference's in-tree CylinderFlow mesh, decoded once and committed as data
    (tests/golden/cylinder_mesh.npz: pos, triangles, 6 velocity frames, node types)."""
    path = path or os.path.join(repo_root(), "tests", "golden", "cylinder_mesh.npz")
    z = np.load(path)
    return {k: z[k] for k in z.files}


def cylinder_batch(batch, t=0, jitter=0.0, seed=1234, mesh=None):
    """B block-diagonal copies of the CylinderFlow mesh as a training sample:
    x=[vx, vy, node_type] [N,3], y = next-frame velocity [N,2], edge_index [2,E] int64 (sorted),
    edge_attr [E,3], pos [N,2]. Optional seeded ±jitter on positions so copies differ."""
    m = mesh or load_cylinder_mesh()
    pos0, tri, vel, nt = m["pos"], m["triangles"], m["velocity"], m["node_type"]
    n = pos0.shape[0]
    ei0 = triangles_to_edge_index(tri, n)
    rng = np.random.default_rng(seed)
    xs, ys, eis, eas, ps = [], [], [], [], []
    for b in range(batch):
        pos = pos0
        if jitter:
            pos = (pos0 * (1.0 + rng.uniform(-jitter, jitter, pos0.shape))).astype(np.float32)
        tt = (t + b) % (vel.shape[0] - 1)
        xs.append(np.concatenate([vel[tt], nt[:, None].astype(np.float32)], 1))
        ys.append(vel[tt + 1])
        eis.append(ei0 + b * n)
        eas.append(edge_features(pos, ei0))
        ps.append(pos)
    return {
        "x": np.concatenate(xs, 0).astype(np.float32),
        "y": np.concatenate(ys, 0).astype(np.float32),
        "edge_index": np.concatenate(eis, 1).astype(np.int64),
        "edge_attr": np.concatenate(eas, 0).astype(np.float32),
        "pos": np.concatenate(ps, 0).astype(np.float32),
        "num_graphs": batch,
        "nodes_per_graph": n,
    }
