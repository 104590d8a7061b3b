"""On-device graph construction through libmgn (include/mgn.h, csrc/mgn_build.hip).

SURVEY.md §8(f) rows 1 and 4: the integer work that turns a mesh into the edge_index / edge_attr
the MGN kernels consume, on HBM-resident tensors, bit-identical to the reference's index sets:

  face_to_edge          T.FaceToEdge + to_undirected (reference dataset/preprocessing.py:410-431;
                        tetrahedra split as utils/torch_graph.py:171-186)
  coalesce              torch_geometric.utils.to_undirected / torch.sparse coalesce
  k_hop_edge_index      utils/torch_graph.py:16-53 (A_k ← coalesce(A_k + A_k·A) minus self loops)
  edge_features         T.Cartesian(norm=False) ‖ T.Distance(norm=False) (preprocessing.py:16-23),
                        add_world_pos_features (preprocessing.py:143-174)
  radius_pairs          cKDTree.query_pairs(r) + OBSTACLE–NORMAL filter of add_world_edges
                        (preprocessing.py:92-140)

No CPU fallback: every entry point requires HIP tensors (graphphysics._native.require_device).
"""
import ctypes

import torch

from graphphysics import _native as N

MGN_COALESCE_SYMMETRIZE = 1
MGN_COALESCE_DROP_SELF_LOOPS = 2


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 8), dtype=torch.uint8, device=device)


def _i64(t):
    if t.dtype != torch.int64 or not t.is_contiguous():
        t = t.to(torch.int64).contiguous()
    return t


def face_to_edge(face, num_nodes):
    """cells [k, C] (k = 3 triangles, k = 4 tetrahedra; the reference's Data.face / tetra layout) →
    undirected edge_index [2, E], sorted by (row, col), no duplicates."""
    N.require_device(face)
    if face.dim() != 2 or face.size(0) not in (3, 4):
        raise ValueError(f"face must be [3, C] or [4, C], got {tuple(face.shape)}")
    face = _i64(face)
    k, c = face.shape
    m = int(N.lib().mgn_face_to_edge_keys(k, c))
    out = torch.empty(2 * max(m, 1), dtype=torch.int64, device=face.device)
    ws = _ws(N.lib().mgn_coalesce_workspace_bytes(m), face.device)
    ne = ctypes.c_int64()
    N.check(N.lib().mgn_face_to_edge(N.ptr(face), k, c, int(num_nodes), N.ptr(out), ctypes.byref(ne), N.ptr(ws),
                                     ws.numel(), N.stream_ptr(face.device)))
    return out[:2 * ne.value].view(2, ne.value)


def coalesce(edge_index, num_nodes, symmetrize=False, drop_self_loops=False):
    """Sorted-unique edge set ([2, E] int64, sorted by (row, col)); symmetrize=True is
    torch_geometric.utils.to_undirected(edge_index, num_nodes=num_nodes) without attributes."""
    N.require_device(edge_index)
    ei = _i64(edge_index)
    e = ei.size(1)
    m = 2 * e if symmetrize else e
    flags = (MGN_COALESCE_SYMMETRIZE if symmetrize else 0) | (MGN_COALESCE_DROP_SELF_LOOPS if drop_self_loops else 0)
    out = torch.empty(2 * max(m, 1), dtype=torch.int64, device=ei.device)
    ws = _ws(N.lib().mgn_coalesce_workspace_bytes(m), ei.device)
    ne = ctypes.c_int64()
    N.check(N.lib().mgn_coalesce(N.ptr(ei), e, int(num_nodes), flags, N.ptr(out), ctypes.byref(ne), N.ptr(ws),
                                 ws.numel(), N.stream_ptr(ei.device)))
    return out[:2 * ne.value].view(2, ne.value)


def to_undirected(edge_index, num_nodes):
    return coalesce(edge_index, num_nodes, symmetrize=True)


def k_hop_edge_index(edge_index, num_hops, num_nodes):
    """compute_k_hop_edge_index (reference utils/torch_graph.py:16-53) on the device: the sparsity
    pattern of A_k after num_hops−1 rounds of A_k ← A_k + A_k·A with the diagonal removed each round,
    A = coalesce(edge_index). Returned coalesced ([2, E] sorted by (row, col))."""
    N.require_device(edge_index)
    a = coalesce(edge_index, num_nodes)
    ak = a
    dev = a.device
    for _ in range(int(num_hops) - 1):
        ek, ea = ak.size(1), a.size(1)
        ws = _ws(N.lib().mgn_khop_count_workspace_bytes(ek, ea, int(num_nodes)), dev)
        nk = ctypes.c_int64()
        N.check(N.lib().mgn_khop_count(N.ptr(ak), ek, N.ptr(a), ea, int(num_nodes), ctypes.byref(nk), N.ptr(ws),
                                       ws.numel(), N.stream_ptr(dev)))
        ws = _ws(N.lib().mgn_khop_workspace_bytes(nk.value, ek, int(num_nodes)), dev)
        out = torch.empty(2 * max(nk.value, 1), dtype=torch.int64, device=dev)
        ne = ctypes.c_int64()
        N.check(N.lib().mgn_khop_hop(N.ptr(ak), ek, N.ptr(a), ea, int(num_nodes), nk.value, N.ptr(out),
                                     ctypes.byref(ne), N.ptr(ws), ws.numel(), N.stream_ptr(dev)))
        ak = out[:2 * ne.value].view(2, ne.value)
    return ak


def edge_features(pos, edge_index):
    """[pos[row] − pos[col] ‖ ‖pos[row] − pos[col]‖₂] as fp32 [E, dim + 1] (Cartesian(norm=False) ‖
    Distance(norm=False); also add_world_pos_features' two blocks)."""
    N.require_device(pos)
    N.require_device(edge_index)
    p = pos
    if p.dtype != torch.float32 or p.dim() != 2 or p.stride(1) != 1:
        p = p.float().contiguous()
    ei = _i64(edge_index)
    e, dim = ei.size(1), p.size(1)
    out = torch.empty((e, dim + 1), dtype=torch.float32, device=p.device)
    ws = _ws(8, p.device)
    N.check(N.lib().mgn_edge_features(N.ptr(p), p.stride(0), dim, N.ptr(ei), e, p.size(0), N.ptr(out), dim + 1,
                                      N.ptr(ws), ws.numel(), N.stream_ptr(p.device)))
    return out


def radius_pairs(pos, radius, node_type=None):
    """All pairs (i, j), i < j, with ‖pos_i − pos_j‖₂ ≤ radius (fp64 distances, cKDTree.query_pairs
    semantics) as [2, P] int64; with node_type (a float column, e.g. x[:, k]) only OBSTACLE–NORMAL
    pairs in either order are kept (add_world_edges' mask). Pair order is unspecified (the
    reference's is cKDTree's); callers coalesce."""
    N.require_device(pos)
    p = pos
    if p.dtype != torch.float32 or p.dim() != 2 or p.stride(1) != 1:
        p = p.float().contiguous()
    n, dim = p.shape
    nt, ntld = None, 0
    if node_type is not None:
        N.require_device(node_type)
        nt = node_type if node_type.dtype == torch.float32 else node_type.float()
        ntld = nt.stride(0) if nt.dim() == 1 else nt.stride(0)
    ws = _ws(N.lib().mgn_radius_pairs_workspace_bytes(n), p.device)
    npairs = ctypes.c_int64()
    args = (N.ptr(p), p.stride(0), dim, n, float(radius), N.ptr(nt), ntld)
    N.check(N.lib().mgn_radius_pairs(*args, N.ptr(None), 0, ctypes.byref(npairs), N.ptr(ws), ws.numel(),
                                     N.stream_ptr(p.device)))
    cnt = npairs.value
    out = torch.empty(2 * max(cnt, 1), dtype=torch.int64, device=p.device)
    if cnt > 0:
        N.check(N.lib().mgn_radius_pairs(*args, N.ptr(out), cnt, ctypes.byref(npairs), N.ptr(ws), ws.numel(),
                                         N.stream_ptr(p.device)))
    return out[:2 * cnt].view(2, cnt)
