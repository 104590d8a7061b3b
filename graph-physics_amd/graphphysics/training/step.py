"""One MGN training step, optionally captured as a hipGraph.

Semantics = the reference's LightningModule.training_step + Lightning automatic optimisation
(reference graphphysics/training/lightning_module.py:111-122, 275-292): Simulator train forward
(normalizer accumulation, one-hot, EncodeProcessDecode) → masked L2 loss over NORMAL ∪ OUTFLOW
nodes → backward → AdamW → cosine-warmup LR step (scheduler.py:41-67).

Captured mode (single process): the whole forward + backward + AdamW launch sequence (~140 kernels)
is recorded once into a hipGraph and replayed; per step the host only writes {lr, step} to the
device and calls replay(), so host/launch overhead disappears. Requires a static batch (the bench's
resident synthetic meshes, or a training loop that copies each batch into the same buffers).
Data parallel (process group of >1 rank), captured: three exchanges (graphphysics.training.distributed)
— the normalizer batch statistics and the global masked-node count, summed over ranks in ONE packed
all-reduce by Simulator.exchange_statistics() (they depend only on the batch, so exchanging them before
the forward is exact), and the parameter gradients. Over RCCL (backend "nccl") all of it is recorded in
the graph: the statistics launch and its all-reduce, the forward, the backward with the gradient
all-reduce bucketed and overlapped on a communication stream (distributed.GradBuckets: the decoder's
and each block's gradients are all-reduced as soon as the backward has produced them — on the
concurrent processor backward, as soon as the side stream has reduced each block's slabs), and AdamW:
one replay per step. Over gloo (not capturable) the statistics exchange runs before the replay and ONE
all-reduce of the flat gradient buffer + AdamW after it; MGN_GRAD_OVERLAP=0 does the same over RCCL.
`graph=False`: the same exchanges, fully eager.

capture() warms the allocator and the library up with `warmup` eager steps and then RESTORES every
piece of state they touched (parameters, optimizer moments and step count, scheduler, learning rate,
normalizer buffers), so N calls are exactly N reference updates. The captured step owns one flat
gradient buffer; the all-reduce and AdamW always read THAT buffer (re-pointing p.grad at it when
eager() or zero_grad() moved it).

New batches: the loss mask (node types) and, data-parallel, the global masked-node count are taken
from the CURRENT batch every step (the count rides in the statistics all-reduce). A captured step
replays the tensors it recorded: assigning a new batch (`step.batch = b`) copies b's x / y /
edge_attr into them when b shares the recorded edge_index (same tensor, unmodified); any other new
batch is re-captured (a different topology).

Validation errors flagged on libmgn's device error word (out-of-range edge_index, node types outside
the one-hot range) surface as the reference's IndexError / RuntimeError at most one step late,
without a host synchronisation per step. The device predicates the state updates on that word (ABI
v11: no AdamW update, no node / edge normalizer accumulation while an error is pending), and the
raise rewinds the host-side step count and LR schedule by the updates the device skipped, so a loop
that catches the error and skips the batch continues from the state the reference would have.
"""
import os
import time

import torch
import torch.distributed as dist

from graphphysics import _native as nat
from graphphysics.training.distributed import GradBuckets, allreduce_gradients, flat_grad_buffer
from graphphysics.utils.loss import masked_mse
from graphphysics.utils.nodetype import NodeType


_CTL_GROUPS = {}


def control_group(group=None):
    """The host-side (gloo) group TrainStep agrees its per-step re-capture decision on: `group` itself
    when it is a gloo group, else one gloo group over the same ranks, created once per process and rank
    set. dist.new_group is a collective over the default group: the first call for a rank set must be
    made by every rank of the world (ranks outside `group` included)."""
    if dist.get_backend(group) == "gloo":
        return group if group is not None else dist.group.WORLD
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else None
    # cached per rank set AND per default process group: after destroy_process_group() and a
    # re-init (elastic restart, tests) the cached group belongs to a destroyed world and is rebuilt
    world = dist.group.WORLD
    ent = _CTL_GROUPS.get(ranks)
    if ent is None or ent[0] is not world:
        ent = _CTL_GROUPS[ranks] = (world, dist.new_group(ranks=list(ranks) if ranks is not None else None,
                                                          backend="gloo"))
    return ent[1]


class TrainStep:
    def __init__(self, sim, opt, sched, batch, masks=(NodeType.NORMAL, NodeType.OUTFLOW), graph=True,
                 group=None, data_parallel=None):
        self.sim, self.opt, self.sched, self.batch = sim, opt, sched, batch
        self.masks = list(masks)
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        # data_parallel=True forces the exchanging step at any world size (tests run it on 1 rank)
        self.dp = self.world > 1 if data_parallel is None else bool(data_parallel)
        self.params = [p for p in sim.parameters() if p.requires_grad]
        self.use_graph = graph
        self.graph = None
        self.static_loss = None
        self._count = None
        self._graph_grads = None  # p.grad views of the captured step's flat gradient buffer
        self._gflat = None
        # bucketed all-reduce overlapped with the backward, recorded in the graph (RCCL only: gloo
        # collectives run on the host and cannot be captured)
        self.overlap = False
        if self.dp and graph and os.environ.get("MGN_GRAD_OVERLAP", "1") != "0" and dist.is_available() \
                and dist.is_initialized():
            self.overlap = dist.get_backend(group) == "nccl"
        self.buckets = None
        self._static = None  # graph mode: the batch tensors the graph was recorded on
        if self.dp:
            sim.set_process_group(group if group is not None else dist.group.WORLD)
        # captured data-parallel step: every rank must choose the same between copy-then-replay and a
        # re-capture (their collective sequences differ), so the choice is agreed on a host-side (gloo)
        # control group — no device synchronisation, no extra collective on the GPU stream. Creating it
        # is a collective over the default group the first time a rank set is seen (control_group):
        # every rank of the world constructs its TrainStep(s) in the same order, as for any DDP model
        self._ctl = None
        self.ctl_seconds = 0.0  # host time spent in the per-step agreement (bench reports it at N > 1)
        if self.dp and graph and self.world > 1:
            self._ctl = control_group(group)

    @property
    def node_type(self):
        """Node types of the CURRENT batch (the loss mask)."""
        return self.batch.x[:, self.sim.node_type_index]

    def _seed(self, loss):
        """d loss / d loss = 1 from a resident tensor (autograd would launch a fill kernel per step)."""
        one = getattr(self, "_one", None)
        if one is None or one.device != loss.device or one.dtype != loss.dtype:
            one = self._one = torch.ones_like(loss)
        return one

    def _loss(self):
        net, tdn, _ = self.sim(self.batch)
        return masked_mse(tdn, net, self.node_type, self.masks, count=self._count)

    def _prologue(self):
        """Data parallel: this batch's normaliser statistics AND its masked-node count, summed over
        ranks in one all-reduce (every step: the batch may have changed)."""
        if self.dp:
            self._count = self.sim.exchange_statistics(self.batch, self.group, loss_masks=self.masks)

    def _raised(self, ex):
        """A validation error of an earlier step surfaced (reference IndexError / RuntimeError): the
        device skipped every optimizer update since (mgn_adamw_dev predication), so rewind the
        host-side counters by as many. Every poll point of a step comes before its own stage()."""
        n = getattr(ex, "mgn_skipped_updates", 0)
        if n:
            self._rewind(n)
        if self.dp and self.world > 1:
            # data parallelism: the device skipped the update on THIS rank only, the other
            # ranks applied theirs, so the replicas no longer agree; as an exception on one rank of the
            # reference's DDP job ends that job, every later step of this TrainStep refuses to run
            self._dp_diverged = "%s: %s" % (type(ex).__name__, ex)

    def _check_replicas(self):
        if getattr(self, "_dp_diverged", None):
            raise RuntimeError("data-parallel TrainStep after a validation error on this rank (%s): the "
                               "replicas' parameters differ; restart from a checkpoint" % self._dp_diverged)

    def _rewind(self, n):
        for g in self.opt.param_groups:
            if "step_count" in g:
                g["step_count"] = max(g["step_count"] - n, 0)
                for p in g["params"]:
                    st = self.opt.state.get(p)
                    if st is not None and "step" in st:
                        st["step"] = torch.tensor(float(g["step_count"]))
        sc = self.sched
        sc.last_epoch = max(sc.last_epoch - n, 0)
        if hasattr(sc, "get_lr_factor"):  # CosineWarmupScheduler: closed form
            lrs = [b * sc.get_lr_factor(epoch=sc.last_epoch) for b in sc.base_lrs]
        elif hasattr(sc, "_get_closed_form_lr"):  # StepLR, CosineAnnealingLR, ExponentialLR, ...
            lrs = sc._get_closed_form_lr()
        else:
            import warnings

            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                lrs = sc.get_lr()
        for g, lr in zip(self.opt.param_groups, lrs):
            g["lr"] = lr
        sc._last_lr = list(lrs)

    def eager(self):
        self._check_replicas()
        try:
            nat.poll_errors(self.batch.x.device)
            self.opt.zero_grad(set_to_none=True)
            self._prologue()
            loss = self._loss()  # the Simulator / topology build poll the error word too
        except (IndexError, RuntimeError) as ex:
            self._raised(ex)
            raise
        loss.backward(self._seed(loss))
        if self.dp:
            allreduce_gradients(self.params, self.group)
        self.opt.step()
        nat.error_word(self.batch.x.device).arm()  # the copy-back carries the optimizer's skip count
        self.sched.step()
        return loss.detach()  # the backward ran: the caller gets the value, not the autograd graph

    def _snapshot(self):
        """Everything an eager step mutates: parameters + buffers (normalizer accumulators), the
        optimizer's moments / step counts / learning rates, the scheduler."""
        tensors = [t for t in list(self.sim.parameters()) + list(self.sim.buffers())]
        groups = []
        for g in self.opt.param_groups:
            fs = g.get("flat_state")
            groups.append((g.get("step_count"), g["lr"], fs, tuple(t.clone() for t in fs) if fs else None))
        return ([t.detach().clone() for t in tensors], tensors, groups, self.sched.state_dict())

    @torch.no_grad()
    def _restore(self, snap):
        vals, tensors, groups, sched = snap
        for t, v in zip(tensors, vals):
            t.copy_(v)
        for g, (cnt, lr, fs, fsv) in zip(self.opt.param_groups, groups):
            if cnt is None:
                g.pop("step_count", None)
            else:
                g["step_count"] = cnt
            g["lr"] = lr
            cur = g.get("flat_state")
            if cur is not None:
                for t, v in zip(cur, fsv if fsv is not None else (None, None)):
                    t.copy_(v) if v is not None else t.zero_()
            for p in g["params"]:
                st = self.opt.state.get(p)
                if st is not None and "step" in st:
                    st["step"] = torch.tensor(float(cnt or 0))
        self.sched.load_state_dict(sched)

    def capture(self, warmup=2, on_record=None):
        """Run `warmup` eager steps on a side stream (allocator + library state), restore the state
        they changed (so they are not extra updates), then record one step. The graph reads private
        copies of the batch's x / y / edge_attr (later batches are copied into them, never into the
        caller's tensors) and the batch's edge_index itself (its topology is cached per tensor)."""
        from graphphysics.utils.data import Data

        b = self.batch
        dev = b.x.device
        # a validation error of an EARLIER step surfaces here with its real skipped-update count
        try:
            nat.check_errors(dev)
        except (IndexError, RuntimeError) as ex:
            self._raised(ex)
            raise
        extra = {k: getattr(b, k) for k in ("pos",) if getattr(b, k, None) is not None}
        self.batch = Data(x=b.x.clone(), y=b.y.clone(), edge_attr=b.edge_attr.clone(), edge_index=b.edge_index,
                          **extra)
        snap = self._snapshot()
        # the warm-up steps are undone on a bad batch, so is the divergence mark one of them may set
        # (ADVICE r04): the recovery step below must run, and only ITS error marks the replicas
        diverged = getattr(self, "_dp_diverged", None)
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        try:
            with torch.cuda.stream(side):
                for _ in range(max(warmup, 1)):
                    self.eager()
            cur.wait_stream(side)
            torch.cuda.synchronize()
            nat.check_errors(dev)  # the warm-up steps validated THIS batch
        except (IndexError, RuntimeError):
            # the batch is invalid: undo the warm-up steps (their skipped updates and normalizer
            # accumulations are not the caller's), then run ONE eager step on it — exactly what the
            # eager path does with a bad batch (the normalizers the reference runs before its raise
            # accumulate; the device skips the update) — and raise with that step's skip count
            from graphphysics.models import _engine

            torch.cuda.synchronize()
            nat.error_word(dev)._clear()
            self._restore(snap)
            self._dp_diverged = diverged
            self.batch = b
            self.graph = None
            _engine.forget_topology(b.edge_index)  # its cached (clamped) topology would not re-flag it
            self.eager()
            torch.cuda.synchronize()
            try:
                nat.check_errors(dev)
            except (IndexError, RuntimeError) as ex2:
                self._raised(ex2)
                raise
            raise RuntimeError("libmgn: validation error during graph warm-up did not reproduce eagerly")
        self._restore(snap)
        self.opt.zero_grad(set_to_none=True)
        if on_record is not None:
            on_record()
        if not self.overlap:
            self._prologue()  # pending statistics exist before recording (the graph reads their buffers)
        # no fallback: a failure to record the overlapped all-reduce raises on every rank (a rank that
        # silently re-recorded without it would issue a different collective sequence)
        g, loss = self._record()
        # the replay writes the loss into this tensor's storage; detached, it does not keep the recorded
        # autograd graph alive — whose AccumulateGrad nodes carry the capture stream, so an eager step
        # between replays reused them from another stream ("AccumulateGrad node's stream does not match")
        self.graph, self.static_loss = g, loss.detach()
        self._graph_grads = [p.grad for p in self.params]
        self._gflat = flat_grad_buffer(self.params)
        b = self.batch
        self._static = {"batch": b, "x": b.x, "y": b.y, "edge_attr": b.edge_attr, "edge_index": b.edge_index,
                        "ei_version": b.edge_index._version}
        return self

    def _sync_batch(self):
        """Graph mode: the replay reads the tensors it was recorded on. A new batch sharing the
        recorded edge_index is copied into them; any other new batch (or an edge_index modified in
        place: the recorded topology would be stale) is re-captured."""
        st = self._static
        b = self.batch
        if b is st["batch"] and all(getattr(b, k) is st[k] for k in ("x", "y", "edge_attr", "edge_index")) \
                and b.edge_index._version == st["ei_version"]:
            return
        same = b.edge_index is st["edge_index"] and b.edge_index._version == st["ei_version"] and all(
            getattr(b, k).shape == st[k].shape and getattr(b, k).dtype == st[k].dtype for k in ("x", "y", "edge_attr"))
        if same:
            with torch.no_grad():
                for k in ("x", "y", "edge_attr"):
                    if getattr(b, k) is not st[k]:
                        st[k].copy_(getattr(b, k))
            self.batch = st["batch"]
        else:
            self.graph = None  # re-captured on the new batch by __call__

    def _record(self):
        g = torch.cuda.CUDAGraph()
        # with a process group, the RCCL watchdog thread queries its events while this thread records:
        # "global" capture mode would turn that query into hipErrorStreamCaptureUnsupported (abort)
        mode = "thread_local" if dist.is_available() and dist.is_initialized() else "global"
        with torch.cuda.graph(g, capture_error_mode=mode):
            if self.overlap:
                # RCCL: the statistics exchange (one statistics launch, the mask count, ONE all-reduce) is
                # recorded too — it depends only on the batch the graph reads — so a step is ONE replay
                self._prologue()
            loss = self._loss()
            if self.overlap:
                from graphphysics.models import _engine

                mb = float(os.environ.get("MGN_GRAD_BUCKET_MB", "4"))
                self.buckets = GradBuckets(self.group, bucket_bytes=int(mb * (1 << 20)))
                _engine.GRAD_READY = self.buckets
                try:
                    loss.backward(self._seed(loss))
                finally:
                    _engine.GRAD_READY = None
                self.buckets.finish()
                total = sum(p.numel() for p in self.params)
                if self.buckets.covered != total:
                    raise RuntimeError("overlapped gradient all-reduce covered %d of %d gradient elements (the "
                                       "model is not one EncodeProcessDecode): set MGN_GRAD_OVERLAP=0"
                                       % (self.buckets.covered, total))
                self.opt.launch()
            else:
                loss.backward(self._seed(loss))
                if not self.dp:
                    self.opt.launch()
        return g, loss

    def _bind_graph_grads(self):
        """p.grad -> the captured step's gradient buffer (eager() / zero_grad() may have moved it)."""
        gg = self._graph_grads
        if self.params[0].grad is not gg[0] or self.params[-1].grad is not gg[-1]:
            for p, g in zip(self.params, gg):
                p.grad = g

    def __call__(self):
        if not self.use_graph:
            return self.eager()
        self._check_replicas()
        dev = self.batch.x.device
        try:
            nat.poll_errors(dev)
        except (IndexError, RuntimeError) as ex:
            self._raised(ex)
            raise
        if self.graph is not None:
            self._sync_batch()
        if self._ctl is not None:
            # re-capture on every rank if any rank needs to (a rank that copies and
            # replays while another re-captures would pair mismatched collectives)
            t0 = time.perf_counter()
            need = torch.tensor([1 if self.graph is None else 0], dtype=torch.int32)
            dist.all_reduce(need, op=dist.ReduceOp.MAX, group=self._ctl)
            self.ctl_seconds += time.perf_counter() - t0
            if int(need[0]):
                self.graph = None
        if self.graph is None:
            self.capture()
        self._bind_graph_grads()
        self.opt.stage()
        if self.dp and self.overlap:
            self.graph.replay()  # statistics exchange, backward-overlapped gradient all-reduce + AdamW inside
        elif self.dp:
            self._prologue()
            self.graph.replay()
            if self._gflat is not None and dist.is_available() and dist.is_initialized():
                dist.all_reduce(self._gflat, group=self.group)
            else:
                allreduce_gradients(self.params, self.group)
            self.opt.launch()
        else:
            self.graph.replay()
        nat.error_word(dev).arm()
        self.sched.step()
        return self.static_loss
