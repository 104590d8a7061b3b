"""Autoregressive validation rollout on the libmgn inference kernels.

Semantics = the reference's LightningModule validation path:
  build_mask            lightning_module.py:17-25  (nodes that are neither NORMAL nor OUTFLOW keep
                                                    their ground truth)
  _make_prediction      lightning_module.py:168-202 (feed the previous prediction back into
                                                    x[:, output_index_start:end]; optional
                                                    previous-data channel; no_grad forward;
                                                    predicted[mask] = target[mask])
  validation_step loss  lightning_module.py:204-232 (masked L2 over NORMAL ∪ OUTFLOW)
  all-rollout RMSE      lightning_module.py:236-249 (sqrt(mean((pred − target)²)) over every step)
  trajectory reset      lightning_module.py:163-166

The forward runs in no-grad mode, so GraphNetBlocks use mgn_block_forward's inference kernels (no
backward saves). With graph=True the per-step work after the first step of a trajectory — write
the previous prediction into the static input, Simulator eval forward, mask, keep the prediction —
is one hipGraph replay; the host only copies the next frame's x and y into the static buffers.
Masking uses torch.where (the reference's boolean index_put would synchronise with the host). The
graph is re-recorded when the mesh (edge_index) changes.
"""
import math
import weakref

import torch

from graphphysics.utils.loss import masked_mse
from graphphysics.utils.nodetype import NodeType


def build_mask(param, graph):
    """True on nodes whose prediction is replaced by the target (reference lightning_module.py:17-25).
    param: the reference's parameter dict ({"index": {"node_type_index": k}}) or the index itself."""
    k = param["index"]["node_type_index"] if isinstance(param, dict) else int(param)
    node_type = graph.x[:, 0, k] if graph.x.dim() > 2 else graph.x[:, k]
    return torch.logical_not(torch.logical_or(node_type == NodeType.NORMAL, node_type == NodeType.OUTFLOW))


class _Frame:
    """Attribute bag standing in for the cloned PyG batch (x, y, edge_index, edge_attr, pos)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


class Rollout:
    def __init__(self, sim, node_type_index, masks=(NodeType.NORMAL, NodeType.OUTFLOW), use_previous_data=False,
                 previous_data_start=None, previous_data_end=None, graph=True):
        self.sim = sim
        self.k = int(node_type_index)
        self.masks = list(masks)
        self.use_prev = use_previous_data
        self.ps, self.pe = previous_data_start, previous_data_end
        self.use_graph = graph
        self.os, self.oe = sim.output_index_start, sim.output_index_end
        self._graph = None
        self._key = None
        self.outputs, self.targets, self.losses = [], [], []
        self.reset()

    # ------------------------------------------------------------------ trajectory bookkeeping
    def reset(self):
        """Start a new trajectory (reference _reset_validation_trajectory)."""
        self.last_prediction = None
        self.last_previous = None

    def clear(self):
        """Forget recorded steps (reference _reset_validation_epoch_end)."""
        self.outputs.clear()
        self.targets.clear()
        self.losses.clear()
        self.reset()

    # ------------------------------------------------------------------ one step
    def _predict(self, fr, last, last_prev):
        if last is not None:
            fr.x[:, self.os:self.oe] = last
            if self.use_prev:
                fr.x[:, self.ps:self.pe] = last_prev
        mask = build_mask(self.k, fr)
        current = fr.x[:, self.os:self.oe].clone()
        with torch.no_grad():
            _, _, pred = self.sim(fr)
        pred = torch.where(mask[:, None], fr.y, pred)
        prev = pred - current if self.use_prev else None
        return pred, prev

    def _eager(self, batch):
        fr = _Frame(x=batch.x.clone(), y=batch.y, edge_index=batch.edge_index, edge_attr=batch.edge_attr,
                    pos=getattr(batch, "pos", None))
        return self._predict(fr, self.last_prediction, self.last_previous)

    def _record(self, batch):
        dev = batch.x.device
        self._sx, self._sy = batch.x.clone(), batch.y.clone()
        self._sea = batch.edge_attr.clone()
        self._sei = batch.edge_index
        self._last = self.last_prediction.clone()
        self._lastp = self.last_previous.clone() if self.use_prev else None
        fr = _Frame(x=self._sx, y=self._sy, edge_index=self._sei, edge_attr=self._sea, pos=getattr(batch, "pos", None))
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up: topology cache, weight packs, allocator
            self._predict(fr, self._last, self._lastp)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        # the graph reads this topology's buffers: keep them alive beyond the topology cache
        from graphphysics.models import _engine

        self._topo = _engine.get_topology(self._sei, self._sx.size(0))
        self._sx.copy_(batch.x)
        g = torch.cuda.CUDAGraph()
        import torch.distributed as dist

        # a process group's watchdog thread queries events while this thread records (see TrainStep)
        mode = "thread_local" if dist.is_available() and dist.is_initialized() else "global"
        with torch.cuda.graph(g, capture_error_mode=mode):
            pred, prev = self._predict(fr, self._last, self._lastp)
            self._last.copy_(pred)
            if self.use_prev:
                self._lastp.copy_(prev)
        self._graph, self._gpred, self._gprev = g, pred, prev
        self._key = (weakref.ref(batch.edge_index), batch.edge_index._version, batch.x.shape)

    def _same_mesh(self, batch):
        """The recorded graph holds the topology of this exact edge_index tensor (identity + version,
        as graphphysics.models._engine.get_topology) and static buffers of this x shape."""
        if self._key is None:
            return False
        ref, ver, shape = self._key
        return ref() is batch.edge_index and ver == batch.edge_index._version and shape == batch.x.shape

    def step(self, batch):
        """One _make_prediction on `batch` (x, y, edge_index, edge_attr on the device). Returns
        (predicted_outputs, target) and records them and the step's masked L2 loss."""
        if not self.use_graph or self.last_prediction is None:
            pred, prev = self._eager(batch)
        else:
            if self._graph is None or not self._same_mesh(batch):
                self._record(batch)
            else:
                self._sx.copy_(batch.x)
                self._sy.copy_(batch.y)
                self._sea.copy_(batch.edge_attr)
                self._last.copy_(self.last_prediction)
                if self.use_prev:
                    self._lastp.copy_(self.last_previous)
            self._graph.replay()
            pred = self._gpred.clone()
            prev = self._gprev.clone() if self.use_prev else None
        self.last_prediction, self.last_previous = pred, prev
        node_type = batch.x[:, self.k]
        self.outputs.append(pred)
        self.targets.append(batch.y)
        self.losses.append(masked_mse(batch.y, pred, node_type, self.masks))
        return pred, batch.y

    def rollout(self, frames):
        """Run a whole trajectory (iterable of batches); returns the stacked predictions."""
        self.reset()
        return torch.stack([self.step(b)[0] for b in frames])

    def all_rollout_rmse(self):
        p = torch.cat([o.float() for o in self.outputs])
        t = torch.cat([o.float() for o in self.targets])
        return math.sqrt(((p - t) ** 2).mean().item())
