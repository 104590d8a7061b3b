import torch
import torch.nn as nn


class MessagePassing(nn.Module):
    def __init__(self, aggr="add", flow="source_to_target"):
        super().__init__()
        assert aggr == "add" and flow == "source_to_target"

    def propagate(self, edge_index, x=None, edge_attr=None, size=None):
        msg = self.message(edge_attr)
        n_target = size[1] if size is not None else x.size(0)
        idx = edge_index[1].view(-1, 1).expand_as(msg)
        out = msg.new_zeros((n_target, msg.size(1))).scatter_add_(0, idx, msg)
        return self.update(out, x=x)


class TransformerConv(nn.Module):  # placeholder: transformer path is out of scope
    def __init__(self, *a, **k):
        raise NotImplementedError
