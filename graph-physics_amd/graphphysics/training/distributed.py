"""Graph-sharded data parallelism: one process per GPU, each rank collates its own
graphs (block-diagonal batches never share edges), one RCCL exchange per step.

Exact equivalence with the single-process reference step on the union of all ranks' graphs needs
three things the reference never had to do (it runs devices=1, reference train.py:233-236):
  1. Normalizer batch statistics summed across ranks before they are accumulated
     (Simulator.set_process_group → Normalizer._accumulate all-reduce);
  2. the masked-mean loss divided by the GLOBAL masked-node count (global_masked_mse);
  3. parameter gradients SUMMED across ranks — with (2) that is the gradient of the global loss.
Gradients of EncodeProcessDecode live in one flat buffer, so (3) is a single all-reduce.
"""
import torch
import torch.distributed as dist

from graphphysics.utils.loss import _prepare_mask_for_loss, masked_mse


def global_mask_count(node_type, masks, group=None, dtype=torch.float32):
    """Number of loss-masked nodes over all ranks (one tiny all-reduce)."""
    cnt = _prepare_mask_for_loss(node_type[:, None], node_type, masks).to(dtype).sum().reshape(1)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(cnt, group=group)
    return cnt[0]


def global_masked_mse(target, network_output, node_type, masks, group=None, count=None):
    """L2Loss (reference utils/loss.py:28-65) over the union of all ranks' nodes: the local
    contribution Σ_local err² / (N_global · n_out); summed over ranks it is the global masked mean,
    so SUM-all-reduced gradients are the gradients of the single-process loss."""
    if count is None:
        count = global_mask_count(node_type, masks, group, network_output.dtype)
    return masked_mse(target, network_output, node_type, masks, count=count)


def sum_allreduce_hook(process_group, bucket):
    """DistributedDataParallel communication hook that SUMS gradient buckets over ranks (DDP's
    default hook averages them). With global_masked_mse — whose per-rank losses SUM to the global
    masked mean — the summed gradients are exactly the single-process gradients on the union batch;
    averaged ones would be 1/world_size of them. Register it on the Lightning / DDP path:
        ddp_model.register_comm_hook(None, sum_allreduce_hook)
        # Lightning: Trainer(strategy=DDPStrategy(ddp_comm_hook=sum_allreduce_hook), ...)
    """
    group = process_group if process_group is not None else dist.group.WORLD
    fut = dist.all_reduce(bucket.buffer(), group=group, async_op=True).get_future()
    return fut.then(lambda f: f.value()[0])


def flat_grad_buffer(params):
    """The single contiguous tensor all gradients are views of, or None."""
    gs = [p.grad for p in params if p.grad is not None]
    if not gs:
        return None
    st = gs[0].untyped_storage()
    off = gs[0].storage_offset()
    for g in gs:
        if g.untyped_storage().data_ptr() != st.data_ptr() or g.storage_offset() != off \
                or not g.is_contiguous():
            return None
        off += g.numel()
    n = off - gs[0].storage_offset()
    return torch.empty(0, dtype=gs[0].dtype, device=gs[0].device).set_(st, gs[0].storage_offset(), (n,))


def allreduce_gradients(params, group=None, op=None):
    """Sum gradients over ranks (one collective when they share a flat buffer)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    op = op if op is not None else dist.ReduceOp.SUM
    params = list(params)
    flat = flat_grad_buffer(params)
    if flat is not None:
        dist.all_reduce(flat, op=op, group=group)
        return
    gs = [p.grad for p in params if p.grad is not None]
    buf = torch.cat([g.reshape(-1) for g in gs])
    dist.all_reduce(buf, op=op, group=group)
    o = 0
    for g in gs:
        g.copy_(buf[o:o + g.numel()].view_as(g))
        o += g.numel()


class GradBuckets:
    """Bucketed gradient all-reduce overlapped with the backward ("bucket it and
    overlap it with the backward of later blocks"). Installed as graphphysics.models._engine.GRAD_READY
    while the step's backward is recorded: each call hands over a flat-gradient range that is final
    on the compute stream; adjacent ranges (the processor blocks arrive last-first, each right below
    the previous one) merge into one bucket until it holds `bucket_bytes`, then the bucket is
    SUM-all-reduced in place on a communication stream that waits only for the work that produced
    it. finish() flushes the last bucket and joins the communication stream back into the compute
    stream. Every rank issues the same buckets in the same order (the backward is deterministic), as
    RCCL requires. Inside a hipGraph capture the collectives are recorded into the graph: one replay
    then covers forward, backward, the overlapped all-reduces and the optimizer.

    A range is final on the stream that is CURRENT when it is handed over — the compute stream, or
    the side stream of the concurrent processor backward, whose weight-gradient launches and slab
    reductions run beside the next block's data gradients (models/_engine.py). Each hand-over records
    an event there, and a bucket's collective waits for the events of every range in it, so a bucket
    merging ranges from both streams waits for exactly their producers."""

    def __init__(self, group=None, bucket_bytes=4 << 20):
        self.group = group
        self.bucket = int(bucket_bytes)
        self.comm = None
        self.cur = None  # (G, lo, hi)
        self.events = {}  # open bucket: the latest hand-over event per producer stream
        self.issued = 0
        self.covered = 0  # elements handed over (TrainStep checks they are the whole buffer)

    def __call__(self, G, lo, hi):
        self.covered += hi - lo
        if self.cur is not None and self.cur[0] is G and hi == self.cur[1] \
                and (self.cur[2] - lo) * G.element_size() <= self.bucket:
            self.cur = (G, lo, self.cur[2])
        else:
            self._flush()
            self.cur = (G, lo, hi)
        st = torch.cuda.current_stream(G.device)
        ev = torch.cuda.Event()
        ev.record(st)
        self.events[st.cuda_stream] = ev  # a later event on a stream covers the earlier ones
        if (self.cur[2] - self.cur[1]) * G.element_size() >= self.bucket:
            self._flush()

    def _flush(self):
        if self.cur is None:
            return
        G, lo, hi = self.cur
        self.cur = None
        if self.comm is None:
            self.comm = torch.cuda.Stream(device=G.device)
        for ev in self.events.values():
            self.comm.wait_event(ev)
        self.events = {}
        with torch.cuda.stream(self.comm):
            self._reduce(G[lo:hi])
        self.issued += 1

    def _reduce(self, t):
        """The in-place collective of one bucket, issued on the communication stream."""
        dist.all_reduce(t, group=self.group)

    def finish(self):
        self._flush()
        if self.comm is not None:
            torch.cuda.current_stream(self.comm.device).wait_stream(self.comm)
