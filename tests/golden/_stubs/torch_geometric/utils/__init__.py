"""Import-only placeholder (tests/golden/make_graph_golden.py); never called."""


def to_undirected(*a, **k):
    raise NotImplementedError("torch_geometric.utils placeholder")
