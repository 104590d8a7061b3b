"""Graph container. Uses torch_geometric.data.Data when installed (reference
graphphysics/models/simulator.py:7); otherwise a minimal attribute bag with the fields the MGN
path reads (x, edge_index, edge_attr, pos, y)."""
try:  # pragma: no cover - PyG is not installed in this image
    from torch_geometric.data import Data  # noqa: F401
except ImportError:  # pragma: no cover
    class Data:
        def __init__(self, **kw):
            for k, v in kw.items():
                setattr(self, k, v)

        @property
        def num_nodes(self):
            for k in ("x", "pos"):
                if getattr(self, k, None) is not None:
                    return getattr(self, k).size(0)
            return None

        def to(self, device):
            for k, v in list(vars(self).items()):
                if hasattr(v, "to"):
                    setattr(self, k, v.to(device))
            return self
