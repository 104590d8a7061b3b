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


OBSTACLE, HANDLE = 1, 3  # reference graphphysics/utils/nodetype.py


def tet_grid(nx, ny, nz, spacing, origin=(0.0, 0.0, 0.0)):
    """Structured tetrahedral mesh of an nx × ny × nz node grid: each cube split into the 6 Kuhn
    tetrahedra around its main diagonal. Returns pos [N,3] float32, cells [6·cubes, 4] int64."""
    ii, jj, kk = np.meshgrid(np.arange(nx), np.arange(ny), np.arange(nz), indexing="ij")
    pos = np.stack([ii, jj, kk], -1).reshape(-1, 3) * spacing + np.asarray(origin)
    vid = lambda i, j, k: (i * ny + j) * nz + k  # noqa: E731
    i, j, k = [a.reshape(-1) for a in np.meshgrid(np.arange(nx - 1), np.arange(ny - 1), np.arange(nz - 1),
                                                   indexing="ij")]
    v = {(a, b, c): vid(i + a, j + b, k + c) for a in (0, 1) for b in (0, 1) for c in (0, 1)}
    tets = [(v[0, 0, 0], v[1, 0, 0], v[1, 1, 0], v[1, 1, 1]), (v[0, 0, 0], v[1, 0, 0], v[1, 0, 1], v[1, 1, 1]),
            (v[0, 0, 0], v[0, 1, 0], v[1, 1, 0], v[1, 1, 1]), (v[0, 0, 0], v[0, 1, 0], v[0, 1, 1], v[1, 1, 1]),
            (v[0, 0, 0], v[0, 0, 1], v[1, 0, 1], v[1, 1, 1]), (v[0, 0, 0], v[0, 0, 1], v[0, 1, 1], v[1, 1, 1])]
    cells = np.concatenate([np.stack(t, 1) for t in tets], 0)
    return pos.astype(np.float32), cells.astype(np.int64)


def plate_sample(seed=0, nx=25, ny=13, nz=4, spacing=0.04):
    """DeformingPlate-shaped frame pair (SURVEY.md §8 Cfg C; the dataset is not in-tree): a tet-meshed
    plate (nx·ny·nz nodes, the x = 0 face HANDLE, the rest NORMAL) and a small tet-meshed OBSTACLE
    block 0.02 above its top face, pressing down. Raw layout of the reference's plate frames before
    preprocessing: x = [world_pos(3), node_type], y = next world_pos, pos = mesh_pos, cells [F, 4].
    With build_preprocessing(world_pos_parameters={0, 3, node_type_index 6}) this gives the model's
    node_in 6 + 9, edge_in 3 + 1 + 3 + 1 = 8 (plate.json indices, preprocessing.py:49-174)."""
    rng = np.random.default_rng(seed)
    ppos, pcells = tet_grid(nx, ny, nz, spacing)
    top = ppos[:, 2].max()
    cx, cy = ppos[:, 0].mean(), ppos[:, 1].mean()
    opos, ocells = tet_grid(5, 5, 2, 0.02, origin=(cx - 0.04, cy - 0.04, top + 0.02))
    n_p = ppos.shape[0]
    mesh_pos = np.concatenate([ppos, opos], 0)
    cells = np.concatenate([pcells, ocells + n_p], 0)
    nt = np.full(mesh_pos.shape[0], NORMAL, np.float32)
    nt[:n_p][ppos[:, 0] == 0] = HANDLE
    nt[n_p:] = OBSTACLE
    # current world positions: a small seeded bend of the plate; next frame: the obstacle moves down,
    # plate nodes follow with a smooth displacement, handles stay
    world = mesh_pos.copy()
    world[:n_p, 2] += 0.005 * np.sin(np.pi * ppos[:, 0] / ppos[:, 0].max()) * rng.uniform(0.5, 1.5)
    nxt = world.copy()
    nxt[n_p:, 2] -= 0.003
    r = np.hypot(world[:n_p, 0] - cx, world[:n_p, 1] - cy)
    nxt[:n_p, 2] -= 0.002 * np.exp(-(r / 0.1) ** 2) * (nt[:n_p] == NORMAL)
    nxt[:n_p] += 1e-4 * rng.standard_normal((n_p, 3)) * (nt[:n_p, None] == NORMAL)
    x = np.concatenate([world, nt[:, None]], 1).astype(np.float32)
    return {"x": x, "y": nxt.astype(np.float32), "pos": mesh_pos.astype(np.float32), "cells": cells}


def plate_graph(device, seed=0, **kw):
    """plate_sample() through the reference's DeformingPlate preprocessing on the device
    (build_preprocessing with world_pos_parameters {0, 3, node_type_index 6}, plate.json:17-37):
    add_obstacles_next_pos → FaceToEdge (tetrahedra) → world edges (r = 0.03) → Cartesian + Distance
    → relative world-pos features. Returns (Data with x [N, 7] = [world(3), disp(3), type],
    y [N, 3], edge_index, edge_attr [E, 8]; the Simulator layout dict)."""
    import torch

    from graphphysics.dataset.preprocessing import build_preprocessing
    from graphphysics.utils.data import Data

    s = plate_sample(seed=seed, **kw)
    d = Data(x=torch.from_numpy(s["x"]).to(device), y=torch.from_numpy(s["y"]).to(device),
             pos=torch.from_numpy(s["pos"]).to(device),
             face=torch.from_numpy(s["cells"]).t().contiguous().to(device))
    g = build_preprocessing(world_pos_parameters={"world_pos_index_start": 0, "world_pos_index_end": 3,
                                                  "node_type_index": 6})(d)
    g.face = None
    lay = dict(node_in=15, edge_in=8, out=3, fs=(0, 6), os=(0, 3), nti=6)
    return g, lay
