"""Import-only placeholder for meshio (used ONLY by tests/golden/make_graph_golden.py so that the
reference's graphphysics/utils/torch_graph.py imports; nothing here is ever called)."""


class Mesh:
    def __init__(self, *a, **k):
        raise NotImplementedError("meshio placeholder")
