"""ORACLE — test infrastructure only. CPU restatement of the reference's mesh → graph construction
(SURVEY.md §8(f) rows 1 and 4). Only tests/ may import this module, as the checker of libmgn's
on-device graph construction (graphphysics.utils.graph_build) — never as the product path.

Restated from (reference = cviviers/graph-physics @ /root/reference; torch-geometric 2.6.1 and
scipy are its third-party dependencies, requirements.txt:7):
  face_to_edge        T.FaceToEdge (PyG 2.6.1: pairs face[:2], face[1:], face[::2], then
                      to_undirected), as the reference composes it in
                      graphphysics/dataset/preprocessing.py:410,431
  tetra_faces         graphphysics/utils/torch_graph.py:171-181 (4 triangles per tetrahedron)
  to_undirected       torch_geometric.utils.to_undirected: cat both directions, coalesce
                      (sort by row·N + col, drop duplicates)
  k_hop_edge_index    graphphysics/utils/torch_graph.py:16-53, with the same torch.sparse ops
  edge_features       T.Cartesian(norm=False) ‖ T.Distance(norm=False) (preprocessing.py:16-23;
                      sign pos[row] − pos[col], unpinned offline) and
                      add_world_pos_features (preprocessing.py:143-174)
  world_edges         add_world_edges (preprocessing.py:92-140): scipy cKDTree.query_pairs, the
                      OBSTACLE–NORMAL mask, cat with the mesh edges, to_undirected

Pins (tests/test_graph_oracle.py): edge counts from the reference's own tests (CylinderFlow mock
mesh 11070 edges, 32638 at k-hop 2: tests/graphphysics/dataset/test_xdmfdataset.py:173-175,
228-230) and golden k-hop vectors produced by the reference's compute_k_hop_edge_index itself
(tests/golden/make_graph_golden.py → tests/golden/graph_golden.npz).
"""
import numpy as np
import torch

OBSTACLE, NORMAL = 1, 0


def coalesce_pattern(row, col, n):
    """Sorted unique (row, col) pairs — torch_geometric.utils.coalesce on an index-only graph."""
    key = torch.unique(row.long() * n + col.long())  # sorted
    return torch.stack([key // n, key % n], 0)


def to_undirected(edge_index, n):
    r, c = edge_index[0], edge_index[1]
    return coalesce_pattern(torch.cat([r, c]), torch.cat([c, r]), n)


def tetra_faces(cells):
    """[4, C] tetrahedra → [3, 4C] triangles in the reference's order."""
    c = cells
    return torch.cat([c[0:3], c[1:4], torch.stack([c[2], c[3], c[0]], 0), torch.stack([c[3], c[0], c[1]], 0)], 1)


def face_to_edge(face, n):
    if face.size(0) == 4:
        face = tetra_faces(face)
    ei = torch.cat([face[:2], face[1:], face[::2]], dim=1)
    return to_undirected(ei, n)


def k_hop_edge_index(edge_index, num_hops, n):
    """The reference's sparse recurrence: A_k ← coalesce(A_k + A_k @ A), diagonal entries removed."""
    a = torch.sparse_coo_tensor(edge_index, torch.ones(edge_index.size(1)), (n, n)).coalesce()
    ak = a.clone()
    for _ in range(num_hops - 1):
        ak = (ak + torch.sparse.mm(ak, a)).coalesce()
        idx = ak.indices()
        keep = idx[0] != idx[1]
        ak = torch.sparse_coo_tensor(idx[:, keep], ak.values()[keep], ak.size()).coalesce()
    return ak.indices()


def edge_features(pos, edge_index):
    d = pos[edge_index[0]] - pos[edge_index[1]]
    return torch.cat([d, torch.norm(d, p=2, dim=-1, keepdim=True)], dim=-1)


def radius_pairs(pos, radius):
    from scipy.spatial import cKDTree

    pairs = cKDTree(pos.cpu().numpy()).query_pairs(radius, output_type="ndarray")
    return torch.from_numpy(pairs.T.astype(np.int64).reshape(2, -1))


def world_edges(world_pos, node_type, edge_index, radius):
    added = radius_pairs(world_pos, radius)
    t0, t1 = node_type[added[0]], node_type[added[1]]
    mask = ((t0 == OBSTACLE) & (t1 == NORMAL)) | ((t0 == NORMAL) & (t1 == OBSTACLE))
    return to_undirected(torch.cat([added[:, mask], edge_index], 1), world_pos.size(0))


def pattern_digest(edge_index):
    """Order-sensitive checksum of an int64 [2, E] edge list (sha256 of its little-endian bytes)."""
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(edge_index.cpu().numpy().astype("<i8")).tobytes()).hexdigest()
