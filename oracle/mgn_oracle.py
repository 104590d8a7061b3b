"""ORACLE — test infrastructure only. CPU (pure PyTorch, fp32) restatement of the reference's
MeshGraphNet training path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module, and only as the checker / CPU baseline — never as the product path.

Parity pin: tests/test_oracle_golden.py checks this restatement BIT-EXACTLY against golden
vectors produced by running the reference's own code (tests/golden/make_golden.py).

Restated from (reference = cviviers/graph-physics @ /root/reference):
  rmsnorm              graphphysics/models/layers.py:49-74  (p=-1, eps added outside the sqrt)
  mlp                  graphphysics/models/layers.py:77-113 (Linear,ReLU x (L-1), Linear, [RMSNorm])
  graph_net_block      graphphysics/models/layers.py:667-746 + torch-geometric 2.6.1 propagate
                       (sum over edge_index[1], dim_size = x.size(0))
  encode_process_decode graphphysics/models/processors.py:111-137
  Normalizer           graphphysics/models/layers.py:315-375
  simulator preamble   graphphysics/models/simulator.py:206-290, 292-307, 309-347
  l2_loss              graphphysics/utils/loss.py:10-65
  lr factor            graphphysics/utils/scheduler.py:55-67
The op sequence mirrors the ATen ops the reference dispatches (index, cat, addmm, scatter_add_,
norm/div/mul) so that CPU fp32 results are identical bit for bit.
"""
import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

NODE_TYPE_SIZE = 9
NORMAL, OUTFLOW = 0, 5


# --------------------------------------------------------------------------- functional core
def rmsnorm(x, scale, eps=1e-8):
    r = x.norm(2, dim=-1, keepdim=True) * (x.shape[-1] ** (-0.5))
    return scale * (x / (r + eps))


def mlp(x, p, prefix, n_linear=4, norm=True, masks=None, record=None):
    """p: state-dict-like mapping; linears at Sequential indices 0,2,4,...; RMSNorm at 2L-1.
    masks (test infrastructure, mask-pinned parity): {prefix: [bool [rows, h] per hidden layer]} — the
    ReLU of hidden layer i becomes h * masks[prefix][i] (the same function on the branch those masks
    select: identical to relu wherever the mask equals (h > 0)). record: {prefix: [pre-activations]}."""
    h = x
    pin = masks.get(prefix) if masks is not None else None
    for i in range(n_linear):
        h = F.linear(h, p[f"{prefix}.{2 * i}.weight"], p[f"{prefix}.{2 * i}.bias"])
        if i < n_linear - 1:
            if record is not None:
                record.setdefault(prefix, []).append(h.detach())
            h = h * pin[i].to(h.dtype) if pin is not None else torch.relu(h)
    if norm:
        h = rmsnorm(h, p[f"{prefix}.{2 * n_linear - 1}.scale"])
    return h


def graph_net_block(x, edge_index, e, p, prefix="", masks=None, record=None):
    row, col = edge_index[0], edge_index[1]
    m = mlp(torch.cat([e, x[col], x[row]], dim=-1), p, prefix + "edge_block", masks=masks, record=record)
    aggr = m.new_zeros((x.size(0), m.size(1))).scatter_add_(
        0, col.view(-1, 1).expand_as(m), m)
    upd = mlp(torch.cat([x, aggr], dim=-1), p, prefix + "node_block", masks=masks, record=record)
    e_new = e + m  # residual order as layers.py:698-699 (edge first: autograd accumulation order)
    return x + upd, e_new


def encode_process_decode(graph_x, edge_index, graph_e, p, mp, only_processor=False, masks=None, record=None):
    """masks / record: see mlp (mask-pinned parity checks; default: the reference's ReLUs)."""
    kw = dict(masks=masks, record=record)
    if only_processor:
        x, e = graph_x, graph_e
    else:
        x = mlp(graph_x, p, "nodes_encoder", **kw)
        e = mlp(graph_e, p, "edges_encoder", **kw)
    for b in range(mp):
        x, e = graph_net_block(x, edge_index, e, p, f"processor_list.{b}.", **kw)
    if only_processor:
        return x
    return mlp(x, p, "decode_module", norm=False, **kw)


# --------------------------------------------------------------------------- module form
def _seq_mlp(i, h, o, n_linear=4, norm=True):
    layers = [nn.Linear(i, h), nn.ReLU()]
    for _ in range(n_linear - 2):
        layers += [nn.Linear(h, h), nn.ReLU()]
    layers.append(nn.Linear(h, o))
    if norm:
        layers.append(_Scale(o))
    return nn.Sequential(*layers)


class _Scale(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.scale = nn.Parameter(torch.ones(d))


class _Block(nn.Module):
    def __init__(self, h):
        super().__init__()
        self.edge_block = _seq_mlp(3 * h, h, h)
        self.node_block = _seq_mlp(2 * h, h, h)


class OracleEPD(nn.Module):
    """Parameter container with the reference's state_dict keys and RNG consumption order
    (processors.py:71-109: nodes_encoder, edges_encoder, decode_module, processor_list)."""

    def __init__(self, message_passing_num, node_input_size, edge_input_size, output_size,
                 hidden_size=128, only_processor=False):
        super().__init__()
        self.mp = message_passing_num
        self.only_processor = only_processor
        if not only_processor:
            self.nodes_encoder = _seq_mlp(node_input_size, hidden_size, hidden_size)
            self.edges_encoder = _seq_mlp(edge_input_size, hidden_size, hidden_size)
            self.decode_module = _seq_mlp(hidden_size, hidden_size, output_size, norm=False)
        self.processor_list = nn.ModuleList([_Block(hidden_size) for _ in range(self.mp)])

    def forward(self, x, edge_index, edge_attr):
        p = dict(self.named_parameters())
        return encode_process_decode(x, edge_index, edge_attr, p, self.mp, self.only_processor)


class OracleNormalizer:
    """layers.py:265-375, state held as plain tensors."""

    def __init__(self, size, max_accumulations=10 ** 5, std_epsilon=1e-8):
        self.max_acc = max_accumulations
        self.eps = torch.tensor(std_epsilon, dtype=torch.float32)
        self.acc_count = torch.tensor(0.0)
        self.num_acc = torch.tensor(0.0)
        self.acc_sum = torch.zeros((1, size))
        self.acc_sum_squared = torch.zeros((1, size))

    def __call__(self, data, accumulate=True):
        if accumulate and self.num_acc < self.max_acc:
            d = data.detach()
            self.acc_sum += torch.sum(d, dim=0, keepdim=True)
            self.acc_sum_squared += torch.sum(d ** 2, dim=0, keepdim=True)
            self.acc_count += d.shape[0]
            self.num_acc += 1
        return (data - self.mean()) / self.std()

    def inverse(self, data):
        return data * self.std() + self.mean()

    def mean(self):
        return self.acc_sum / torch.max(self.acc_count, torch.tensor(1.0))

    def std(self):
        c = torch.max(self.acc_count, torch.tensor(1.0))
        var = self.acc_sum_squared / c - self.mean() ** 2
        return torch.max(torch.sqrt(torch.clamp(var, min=0.0)), self.eps)


class OracleSimulator:
    """simulator.py:128-347 for the CylinderFlow index layout (features 0:2, type at 2)."""

    def __init__(self, model, node_input_size, edge_input_size, output_size,
                 feature_slice=(0, 2), output_slice=(0, 2), node_type_index=2):
        self.model = model
        self.fs, self.os, self.nti = feature_slice, output_slice, node_type_index
        self.out_norm = OracleNormalizer(output_size)
        self.node_norm = OracleNormalizer(node_input_size)
        self.edge_norm = OracleNormalizer(edge_input_size)

    def forward(self, x, y, edge_index, edge_attr, training=True):
        pre = x[:, self.os[0]:self.os[1]]
        tdn = self.out_norm(y - pre, training)
        onehot = F.one_hot(torch.squeeze(x[:, self.nti].long()), NODE_TYPE_SIZE)
        nf = torch.cat([x[:, self.fs[0]:self.fs[1]], onehot], dim=1)
        nfn = self.node_norm(nf, training)
        ean = self.edge_norm(edge_attr, training)
        net = self.model(nfn, edge_index, ean)
        outputs = None if training else pre + self.out_norm.inverse(net)
        return net, tdn, outputs


def l2_loss(target, out, node_type, masks=(NORMAL, OUTFLOW)):
    mask = node_type == masks[0]
    for mk in masks[1:]:
        mask = torch.logical_or(mask, node_type == mk)
    return torch.mean(((out - target) ** 2)[mask])


def lr_factor(step_index, warmup, max_iters, min_lr_factor=1e-3):
    """scheduler.py:55-67 with epoch = last_epoch + 1."""
    ep = step_index + 1
    f = 0.5 * (1 + np.cos(np.pi * ep / max_iters))
    if ep <= warmup:
        f *= ep * 1.0 / warmup
    return max(f, min_lr_factor)


def train_step_flops(n, e, mp, h, node_in, edge_in, out):
    """forward FLOPs x3 for fwd+bwd (elementwise excluded)."""
    f = mp * (12 * h * h * e + 10 * h * h * n)
    f += 2 * (edge_in * h + 3 * h * h) * e + 2 * (node_in * h + 3 * h * h) * n
    f += 2 * (3 * h * h + h * out) * n
    return 3 * f


__all__ = [
    "rmsnorm", "mlp", "graph_net_block", "encode_process_decode", "OracleEPD",
    "OracleNormalizer", "OracleSimulator", "l2_loss", "lr_factor", "train_step_flops",
]
