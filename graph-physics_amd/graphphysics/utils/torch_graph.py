"""Drop-in mesh → graph helpers (reference graphphysics/utils/torch_graph.py).

  compute_k_hop_edge_index   torch_graph.py:16-53   k-hop pattern on the device (libmgn)
  compute_k_hop_graph        torch_graph.py:56-112  + Cartesian/Distance/world-pos edge features
  meshdata_to_graph          torch_graph.py:115-195 points/cells/point_data → Data (host arrays to
                                                    tensors; tetrahedra split into 4 triangles)

compute_k_hop_edge_index differs from the reference only in where it runs: the reference builds a
torch.sparse COO matrix on `device` (cpu in its tests) and multiplies; here the same sparsity
pattern comes from libmgn's CSR expansion + radix-sort coalesce on the HIP device, so
edge_index must be a HIP tensor (no CPU fallback). num_hops == 1 returns the input unchanged,
like the reference's compute_k_hop_graph.
"""
from functools import partial
from typing import Dict, Optional, Union

import numpy as np
import torch

from graphphysics import transforms as T
from graphphysics.dataset.preprocessing import add_world_pos_features
from graphphysics.utils import graph_build as G
from graphphysics.utils.data import Data


def compute_k_hop_edge_index(edge_index: torch.Tensor, num_hops: int, num_nodes: int) -> torch.Tensor:
    return G.k_hop_edge_index(edge_index, num_hops, num_nodes)


def compute_k_hop_graph(graph, num_hops: int, add_edge_features_to_khop: bool = False, device: str = "cpu",
                        world_pos_index_start: int = 0, world_pos_index_end: int = 3):
    if num_hops == 1:
        return graph
    khop = compute_k_hop_edge_index(graph.edge_index, num_hops, graph.num_nodes)
    g = Data(x=graph.x, edge_index=khop, pos=graph.pos, y=getattr(graph, "y", None),
             face=getattr(graph, "face", None))
    if add_edge_features_to_khop:
        ts = [T.Cartesian(norm=False), T.Distance(norm=False)]
        if world_pos_index_start is not None and world_pos_index_end is not None:
            ts.append(partial(add_world_pos_features, world_pos_index_start=world_pos_index_start,
                              world_pos_index_end=world_pos_index_end))
        g = T.Compose(ts)(g)
    return g


def meshdata_to_graph(points: np.ndarray, cells: np.ndarray, point_data: Optional[Dict[str, np.ndarray]],
                      time: Union[int, float] = 1, target: Optional[Dict[str, np.ndarray]] = None,
                      return_only_node_features: bool = False, id: Optional[str] = None):
    if point_data is not None:
        if any(d.ndim > 1 for d in point_data.values()):
            nf = np.hstack([d for d in point_data.values()] + [np.full((len(points),), time).reshape((-1, 1))])
        else:
            nf = np.vstack([d for d in point_data.values()] + [np.full((len(points),), time)]).T
        node_features = torch.tensor(nf, dtype=torch.float32)
    else:
        node_features = torch.zeros((len(points), 1), dtype=torch.float32)
    if return_only_node_features:
        return node_features
    target_features = None
    if target is not None:
        if any(d.ndim > 1 for d in target.values()):
            tf = np.hstack([d for d in target.values()])
        else:
            tf = np.vstack([d for d in target.values()]).T
        target_features = torch.tensor(tf, dtype=torch.float32)
    c = torch.tensor(np.asarray(cells).T)
    tetra = None
    face = None
    if c.shape[0] == 4:
        tetra = c
        face = torch.cat([c[0:3], c[1:4], torch.stack([c[2], c[3], c[0]], dim=0),
                          torch.stack([c[3], c[0], c[1]], dim=0)], dim=1)
    if c.shape[0] == 3:
        face = c
    return Data(x=node_features, face=face, tetra=tetra, y=target_features,
                pos=torch.tensor(points, dtype=torch.float32), id=id)
