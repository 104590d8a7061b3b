"""Drop-in graph preprocessing (reference graphphysics/dataset/preprocessing.py) on the device.

Same function names, arguments and Data-in/Data-out contract as the reference; the index work
(FaceToEdge, to_undirected, radius search, edge features) runs in libmgn on the graph's HIP
device (graphphysics.utils.graph_build), the O(N) feature edits as device torch ops.

  add_edge_features        preprocessing.py:16-23
  add_obstacles_next_pos   preprocessing.py:49-89
  add_world_edges          preprocessing.py:92-140  (cKDTree.query_pairs → grid radius search)
  add_world_pos_features   preprocessing.py:143-174
  add_noise                preprocessing.py:177-238
  build_preprocessing      preprocessing.py:369-440 (noise, world-pos and edge-feature stages)

Random3DRotate / compute_min_distance_to_type (augmentation / aneurysm features) are outside the
MGN hot path and are not provided.
"""
import math
from functools import partial
from typing import Callable, List, Optional, Union

import torch

from graphphysics import transforms as T
from graphphysics.utils import graph_build as G
from graphphysics.utils.nodetype import NodeType


def add_edge_features() -> List[Callable]:
    return [T.Cartesian(norm=False), T.Distance(norm=False)]


def _3d_face_to_edge(graph):
    """Quad faces [4, F] → the four triangles the reference forms (preprocessing.py:26-46)."""
    face = graph.face
    graph.face = torch.cat([face[0:3], face[1:4], torch.stack([face[2], face[3], face[0]], dim=0),
                            torch.stack([face[3], face[0], face[1]], dim=0)], dim=1)
    return graph


def add_obstacles_next_pos(graph, world_pos_index_start: int, world_pos_index_end: int, node_type_index: int):
    world_pos = graph.x[:, world_pos_index_start:world_pos_index_end]
    other = graph.x[:, world_pos_index_end:]
    disp = graph.y[:, world_pos_index_start:world_pos_index_end] - world_pos
    # node_type_index refers to the layout after the 3 displacement columns are inserted
    node_type = graph.x[:, node_type_index - 3]
    obst = node_type == NodeType.OBSTACLE
    mean_disp = torch.mean(disp[obst], dim=0)
    disp[~obst] = mean_disp
    graph.x = torch.cat([world_pos, disp, other], dim=1)
    return graph


def add_world_edges(graph, world_pos_index_start: int, world_pos_index_end: int, node_type_index: int,
                    radius: float = 0.03):
    world_pos = graph.x[:, world_pos_index_start:world_pos_index_end]
    added = G.radius_pairs(world_pos, radius, node_type=graph.x[:, node_type_index])
    edge_index = torch.cat([added, graph.edge_index.to(added.dtype)], dim=1)
    graph.edge_index = G.to_undirected(edge_index, graph.x.size(0))
    return graph


def add_world_pos_features(graph, world_pos_index_start: int, world_pos_index_end: int):
    f = G.edge_features(graph.x[:, world_pos_index_start:world_pos_index_end], graph.edge_index)
    graph.edge_attr = torch.cat([graph.edge_attr, f.type_as(graph.edge_attr)], dim=-1)
    return graph


def add_noise(graph, noise_index_start: Union[int, List[int]], noise_index_end: Union[int, List[int]],
              noise_scale: Union[float, List[float]], node_type_index: int, t: Optional[float] = None):
    if isinstance(noise_index_start, int):
        noise_index_start = [noise_index_start]
    if isinstance(noise_index_end, int):
        noise_index_end = [noise_index_end]
    if isinstance(noise_scale, float):
        noise_scale = [noise_scale] * len(noise_index_start)
    if len(noise_index_start) != len(noise_index_end):
        raise ValueError("noise_index_start and noise_index_end must have the same length.")
    if len(noise_scale) != len(noise_index_start):
        raise ValueError("noise_scale must have the same length as noise_index_start and noise_index_end.")
    mask = graph.x[:, node_type_index] != NodeType.NORMAL
    for start, end, scale in zip(noise_index_start, noise_index_end, noise_scale):
        feature = graph.x[:, start:end]
        s = 10 * scale * (1 + math.cos(t * math.pi)) if t is not None else scale
        noise = torch.randn_like(feature) * s
        noise[mask] = 0
        graph.x[:, start:end] = feature + noise
    return graph


def build_preprocessing(noise_parameters: Optional[dict] = None, world_pos_parameters: Optional[dict] = None,
                        add_edges_features: bool = True,
                        extra_node_features: Optional[Union[Callable, List[Callable]]] = None,
                        extra_edge_features: Optional[Union[Callable, List[Callable]]] = None) -> T.Compose:
    pre: List[Callable] = []
    if extra_node_features is not None:
        pre.extend(extra_node_features if isinstance(extra_node_features, list) else [extra_node_features])
    if world_pos_parameters is not None:
        ws, we = world_pos_parameters["world_pos_index_start"], world_pos_parameters["world_pos_index_end"]
        nti = world_pos_parameters["node_type_index"]
        pre.extend([
            partial(add_obstacles_next_pos, world_pos_index_start=ws, world_pos_index_end=we, node_type_index=nti),
            T.FaceToEdge(remove_faces=False),
            partial(add_world_edges, world_pos_index_start=ws, world_pos_index_end=we, node_type_index=nti,
                    radius=world_pos_parameters.get("radius", 0.03)),
        ])
        pre.extend(add_edge_features())
        pre.append(partial(add_world_pos_features, world_pos_index_start=ws, world_pos_index_end=we))
    else:
        pre.append(T.FaceToEdge(remove_faces=False))
        if add_edges_features:
            pre.extend(add_edge_features())
    if noise_parameters is not None:
        # the reference inserts the noise stage after the first transform (preprocessing.py:433-442)
        pre.insert(1, partial(add_noise, noise_index_start=noise_parameters["noise_index_start"],
                           noise_index_end=noise_parameters["noise_index_end"],
                           noise_scale=noise_parameters["noise_scale"],
                           node_type_index=noise_parameters["node_type_index"]))
    if extra_edge_features is not None:
        pre.extend(extra_edge_features if isinstance(extra_edge_features, list) else [extra_edge_features])
    return T.Compose(pre)
