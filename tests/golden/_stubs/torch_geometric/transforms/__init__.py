"""Import-only placeholders (tests/golden/make_graph_golden.py): the reference's preprocessing
module imports these names; the golden generator never calls them."""


class BaseTransform:
    pass


def _absent(*a, **k):
    raise NotImplementedError("torch_geometric.transforms placeholder")


Cartesian = Distance = FaceToEdge = Compose = _absent
