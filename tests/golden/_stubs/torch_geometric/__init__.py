"""Minimal stand-in for torch-geometric 2.6.1 used ONLY by tests/golden/make_golden.py.

It restates the two pieces of PyG the reference's MGN path touches:
  * MessagePassing(aggr="add", flow="source_to_target").propagate:
      msg = self.message(edge_attr); out = zeros[N_target, h].scatter_add_(0, edge_index[1], msg);
      return self.update(out, x=x)
    (PyG 2.6.1 documented contract; call site reference graphphysics/models/layers.py:649,694-696)
  * Data: an attribute bag.
Never shipped, never imported by the product path.
"""
