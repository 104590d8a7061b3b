"""Drop-in counterparts of reference graphphysics/models/layers.py for the MGN path.

Same class names, constructor signatures, attributes and state_dict keys as the reference
(RMSNorm layers.py:18-74, build_mlp 77-113, Normalizer 265-392, GraphNetBlock 630-746), so
reference checkpoints load unchanged. GraphNetBlock.forward runs on libmgn (HIP, gfx950); there
is no CPU fallback. The transformer/GMM components of the reference are out of scope.
"""
import os
from typing import Any, Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from graphphysics import _native as nat
from graphphysics.models import _engine


def default_compute_dtype():
    """fp32 (exact-fp32 MFMA, parity path) unless GRAPHPHYSICS_MGN_DTYPE=bf16."""
    v = os.environ.get("GRAPHPHYSICS_MGN_DTYPE", "fp32").lower()
    return torch.bfloat16 if v in ("bf16", "bfloat16") else torch.float32


class RMSNorm(nn.Module):
    """y = scale * x / (||x||_2 * d^-1/2 + eps)  (reference layers.py:49-74). As a stand-alone
    module it evaluates with torch ops; inside build_mlp blocks it is fused into the kernels."""

    def __init__(self, d: int, p: float = -1.0, eps: float = 1e-8, bias: bool = False):
        super().__init__()
        self.d, self.p, self.eps, self.bias = d, p, eps, bias
        self.scale = nn.Parameter(torch.ones(d))
        if self.bias:
            self.offset = nn.Parameter(torch.zeros(d))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.p < 0.0 or self.p > 1.0:
            nrm, dx = x.norm(2, dim=-1, keepdim=True), self.d
        else:
            k = int(self.d * self.p)
            nrm, dx = x[..., :k].norm(2, dim=-1, keepdim=True), k
        y = x / (nrm * dx ** (-0.5) + self.eps)
        return self.scale * y + self.offset if self.bias else self.scale * y


def build_mlp(in_size: int, hidden_size: int, out_size: int, nb_of_layers: int = 4,
              layer_norm: bool = True) -> nn.Module:
    """Linear, ReLU × (L-1), Linear, [RMSNorm] — parameter order/keys as reference layers.py:77-113."""
    assert nb_of_layers >= 2, "The MLP must have at least 2 layers (input and output)."
    mods = [nn.Linear(in_size, hidden_size), nn.ReLU()]
    for _ in range(nb_of_layers - 2):
        mods += [nn.Linear(hidden_size, hidden_size), nn.ReLU()]
    mods.append(nn.Linear(hidden_size, out_size))
    if layer_norm:
        mods.append(RMSNorm(out_size))
    return nn.Sequential(*mods)


class Normalizer(nn.Module):
    """Online feature normaliser (reference layers.py:265-392), same buffers and semantics.

    Differences that do not change results: the `num_accumulations < max_accumulations` test is
    evaluated on device (no host sync per call), and, when `process_group` is set (graph-sharded
    data parallel), the batch statistics are all-reduced before they are accumulated so every rank
    holds the statistics of the global batch."""

    def __init__(self, size: int, max_accumulations: int = 10 ** 5, std_epsilon: float = 1e-8,
                 name: str = "Normalizer", device: Optional[Union[str, torch.device]] = "cuda"):
        super().__init__()
        self.name = name
        self.device = device
        self._max_accumulations = max_accumulations
        self._std_epsilon = torch.tensor(std_epsilon, dtype=torch.float32, requires_grad=False,
                                         device=device)
        self.register_buffer("_acc_count", torch.tensor(0.0, device=device))
        self.register_buffer("_num_accumulations", torch.tensor(0.0, device=device))
        self.register_buffer("_acc_sum", torch.zeros((1, size), dtype=torch.float32, device=device))
        self.register_buffer("_acc_sum_squared",
                             torch.zeros((1, size), dtype=torch.float32, device=device))
        self.process_group = None
        self._pending = None  # (sum, sum_sq, count) of the global batch, set by set_pending()
        self._pending_packed = None  # the same three as one [2*size + 1] tensor (views above)
        self._pending_fresh = False  # refreshed for the next accumulating forward (one-shot)
        self._eps_cache = None

    def batch_statistics(self, d: torch.Tensor):
        """(Σ rows, Σ rows², row count) of one local batch (no exchange)."""
        if d.is_cuda and d.dim() == 2 and 1 <= d.shape[1] <= 32:
            from graphphysics import _native as nat  # batch statistics in one native pass

            s, s2 = nat.column_stats(d.float())
        else:
            s = torch.sum(d, dim=0, keepdim=True)
            s2 = torch.sum(d ** 2, dim=0, keepdim=True)
        return s, s2, torch.full((), float(d.shape[0]), device=d.device)

    def set_pending(self, s, s2, cnt):
        """Statistics (already summed over ranks) that the next accumulating forward uses instead of
        computing and exchanging its own: lets a data-parallel step exchange them before a replayed
        hipGraph. The buffers are static, so a captured forward reads each step's values."""
        if self._pending is None:
            k = s.numel()
            packed = torch.empty(2 * k + 1, dtype=torch.float32, device=s.device)
            self._pending_packed = packed
            self._pending = (packed[:k].view_as(s), packed[k:2 * k].view_as(s2), packed[2 * k])
        self._pending[0].copy_(s)
        self._pending[1].copy_(s2)
        self._pending[2].copy_(cnt.reshape(()))
        self._pending_fresh = True

    def bind_pending(self, packed_view: torch.Tensor):
        """Keep the pending statistics in `packed_view` (float32 [2*size + 1], e.g. a slice of one
        buffer several normalizers share so that a single all-reduce updates them all in place)."""
        k = self._acc_sum.numel()
        self._pending_packed = packed_view
        self._pending = (packed_view[:k].view_as(self._acc_sum), packed_view[k:2 * k].view_as(self._acc_sum_squared),
                         packed_view[2 * k])

    def mark_pending_fresh(self):
        """The bound pending buffer now holds this step's (exchanged) statistics."""
        self._pending_fresh = True

    def clear_pending(self):
        self._pending = None
        self._pending_packed = None
        self._pending_fresh = False

    def _consume_pending(self):
        """Pending statistics feed exactly ONE accumulating forward: a second forward without a new
        exchange would re-add the previous batch's statistics (a hipGraph replay re-reads the bound
        buffer, which its owner refreshes before every replay)."""
        if self._pending is None or (self._pending[0].is_cuda and torch.cuda.is_current_stream_capturing()):
            return
        if not self._pending_fresh:
            raise RuntimeError(f"{self.name}: pending batch statistics were already consumed; exchange "
                               "them (Simulator.exchange_statistics) before every training forward")
        self._pending_fresh = False

    def _eps(self) -> float:
        t = self._std_epsilon
        if self._eps_cache is None or self._eps_cache[0] is not t:
            self._eps_cache = (t, float(t))
        return self._eps_cache[1]

    def _native_ok(self, d: torch.Tensor, accumulate: bool) -> bool:
        if not (d.is_cuda and d.dim() == 2 and 1 <= d.shape[1] <= 32 and not d.requires_grad):
            return False
        if accumulate and self.process_group is not None and self._pending is None:
            return False  # statistics exchanged inside _accumulate: torch path
        bufs = (self._acc_sum, self._acc_sum_squared, self._acc_count, self._num_accumulations)
        return all(b.dtype == torch.float32 and b.is_contiguous() and b.device == d.device for b in bufs)

    def forward(self, batched_data: torch.Tensor, accumulate: bool = True) -> torch.Tensor:
        if accumulate:
            self._consume_pending()
        if self._native_ok(batched_data, accumulate):
            from graphphysics import _native as nat  # one native pass: statistics, _accumulate, normalise

            return nat.normalizer_forward(batched_data.detach(), accumulate,
                                          self._pending_packed if accumulate else None, self._acc_sum,
                                          self._acc_sum_squared, self._acc_count, self._num_accumulations,
                                          float(self._max_accumulations), self._eps())
        if accumulate:
            self._accumulate(batched_data.detach())
        return (batched_data - self._mean()) / self._std_with_epsilon()

    def inverse(self, normalized_batch_data: torch.Tensor) -> torch.Tensor:
        return normalized_batch_data * self._std_with_epsilon() + self._mean()

    def _accumulate(self, d: torch.Tensor):
        if self._pending is not None:
            s, s2, cnt = self._pending
        else:
            s, s2, cnt = self.batch_statistics(d)
        if self.process_group is not None and self._pending is None:
            import torch.distributed as dist

            packed = torch.cat([s.reshape(-1), s2.reshape(-1), cnt.reshape(1)])
            dist.all_reduce(packed, group=self.process_group)
            k = s.numel()
            s, s2, cnt = packed[:k].view_as(s), packed[k:2 * k].view_as(s2), packed[2 * k]
        live = self._num_accumulations < self._max_accumulations
        zero = torch.zeros((), device=d.device)
        self._acc_sum += torch.where(live, s, zero)
        self._acc_sum_squared += torch.where(live, s2, zero)
        self._acc_count += torch.where(live, cnt, zero)
        self._num_accumulations += live.float()

    def _mean(self) -> torch.Tensor:
        return self._acc_sum / self._acc_count.clamp(min=1.0)  # = torch.max(count, 1.0)

    def _std_with_epsilon(self) -> torch.Tensor:
        var = self._acc_sum_squared / self._acc_count.clamp(min=1.0) - self._mean() ** 2
        std = torch.sqrt(torch.clamp(var, min=0.0))
        return torch.max(std, self._std_epsilon.to(std.device))

    def get_variable(self) -> Dict[str, Any]:
        return {
            "_max_accumulations": self._max_accumulations,
            "_std_epsilon": self._std_epsilon,
            "_acc_count": self._acc_count,
            "_num_accumulations": self._num_accumulations,
            "_acc_sum": self._acc_sum,
            "_acc_sum_squared": self._acc_sum_squared,
            "name": self.name,
        }


class GraphNetBlock(nn.Module):
    """MeshGraphNet processor block (reference layers.py:630-746), fused on MI355X.

    forward(x [N,h], edge_index [2,E], edge_attr [E,h]) -> (x', e') with
      m  = edge_block([e ‖ x[col] ‖ x[row]]),  aggr_i = Σ_{col_k = i} m_k,
      x' = x + node_block([x ‖ aggr]),          e' = e + m
    (row = edge_index[0] = source, col = edge_index[1] = target; e' in the caller's edge order).
    """

    def __init__(self, hidden_size: int, nb_of_layers: int = 4, layer_norm: bool = True):
        super().__init__()
        self.edge_block = build_mlp(3 * hidden_size, hidden_size, hidden_size, nb_of_layers, layer_norm)
        self.node_block = build_mlp(2 * hidden_size, hidden_size, hidden_size, nb_of_layers, layer_norm)
        self.compute_dtype = default_compute_dtype()
        self._plan = None

    def _get_plan(self):
        if self._plan is None:
            self._plan = _engine.ModelPlan(self, [self.edge_block, self.node_block], [3, 2])
        return self._plan

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor, edge_attr: torch.Tensor,
                size: int = None) -> Tuple[torch.Tensor, torch.Tensor]:
        nat.require_device(x)
        topo = _engine.get_topology(edge_index, x.size(0))
        plan = self._get_plan()
        return _engine.BlockFunction.apply(plan, nat.mgn_dtype(self.compute_dtype), torch.is_grad_enabled(), x,
                                           edge_attr, topo, *plan.params)
