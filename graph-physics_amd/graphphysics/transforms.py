"""Device-backed stand-ins for the torch_geometric.transforms the reference's preprocessing
composes (reference graphphysics/dataset/preprocessing.py:16-23,369-431; torch-geometric 2.6.1,
not installed here). Same call contract — `transform(data) -> data`, mutating and returning the
graph — but the work runs in libmgn on the graph's HIP device (graphphysics.utils.graph_build):

  FaceToEdge(remove_faces=False)  edge_index = to_undirected(pairs of data.face)
  Cartesian(norm=False, cat=True) edge_attr ‖= pos[row] − pos[col]
  Distance(norm=False, cat=True)  edge_attr ‖= ‖pos[row] − pos[col]‖₂
  Compose(transforms)             sequential application

Only the norm=False forms the reference uses are provided (norm=True raises). Sign convention of
Cartesian: pos[row] − pos[col], the same as the reference's add_world_pos_features
(preprocessing.py:163); PyG 2.6.1's own sign is unpinned offline and the MGN
kernels consume edge_attr as given.
"""
import torch

from graphphysics.utils import graph_build as G


def _num_nodes(data):
    n = getattr(data, "num_nodes", None)
    if n is None:
        for k in ("x", "pos"):
            v = getattr(data, k, None)
            if v is not None:
                return v.size(0)
    return n


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data


class FaceToEdge:
    def __init__(self, remove_faces: bool = True):
        self.remove_faces = remove_faces

    def __call__(self, data):
        face = getattr(data, "face", None)
        if face is not None:
            data.edge_index = G.face_to_edge(face, _num_nodes(data))
            if self.remove_faces:
                data.face = None
        return data


class _PosFeature:
    def __init__(self, norm: bool = False, max_value=None, cat: bool = True):
        if norm:
            raise NotImplementedError("only norm=False (the reference's setting) is implemented")
        self.cat = cat

    def _append(self, data, feat):
        pseudo = getattr(data, "edge_attr", None)
        if pseudo is not None and self.cat:
            pseudo = pseudo.view(-1, 1) if pseudo.dim() == 1 else pseudo
            data.edge_attr = torch.cat([pseudo, feat.type_as(pseudo)], dim=-1)
        else:
            data.edge_attr = feat
        return data


class Cartesian(_PosFeature):
    def __call__(self, data):
        f = G.edge_features(data.pos, data.edge_index)
        return self._append(data, f[:, :-1])


class Distance(_PosFeature):
    def __call__(self, data):
        f = G.edge_features(data.pos, data.edge_index)
        return self._append(data, f[:, -1:])
