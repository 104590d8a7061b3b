"""Execution engine: drives libmgn (include/mgn.h) from PyTorch autograd.

* GraphTopology  — target-sorted edge order + segment pointers for an edge_index (built on device
                   by mgn_topology_build, cached per edge_index tensor object).
* MlpSpec        — one build_mlp nn.Sequential (reference graphphysics/models/layers.py:77-113)
                   seen by the kernels: its Linear weights are packed into MFMA fragments, biases and
                   RMSNorm scale are read straight from the fp32 master parameters.
* ModelPlan      — every MLP of a module in parameter-registration order; one pack launch per
                   forward; gradients land in ONE flat fp32 buffer laid out exactly like
                   module.parameters() (so data-parallel all-reduce and the fused optimizer each
                   touch one contiguous buffer).
* EPDFunction / BlockFunction — torch.autograd.Function wrappers of EncodeProcessDecode.forward
                   (processors.py:111-137) and GraphNetBlock.forward (layers.py:667-701).
Device memory is always allocated here through the PyTorch caching allocator; the library owns
none. No CPU fallback exists: tensors must live on a HIP device.
"""
import ctypes
import os
import weakref

import torch
import torch.nn as nn

from graphphysics import _native as nat


# --------------------------------------------------------------------------- topology
class GraphTopology:
    def __init__(self, edge_index, num_nodes):
        nat.require_device(edge_index)
        L = nat.lib()
        ei = edge_index.to(torch.int64).contiguous()
        if ei.dim() != 2 or ei.shape[0] != 2:
            raise ValueError("edge_index must have shape [2, E]")
        E, N = int(ei.shape[1]), int(num_nodes)
        dev = ei.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.num_nodes, self.num_edges, self.device = N, E, dev
        self.csc_src = torch.empty(max(E, 1), **i32)
        self.csc_dst = torch.empty(max(E, 1), **i32)
        self.csc_eid = torch.empty(max(E, 1), **i32)
        self.row_perm = torch.empty(max(E, 1), **i32)
        self.col_ptr = torch.empty(N + 1, **i32)
        self.row_ptr = torch.empty(N + 1, **i32)
        wsb = L.mgn_topology_workspace_bytes(E, N)
        ws = torch.empty(max(int(wsb), 1), dtype=torch.uint8, device=dev)
        # no host read-back: an out-of-range index is flagged on the device error word (clamped in
        # range meanwhile) and raised as IndexError by the next poll / check_errors()
        ew = nat.error_word(dev)
        ew.poll()
        if E and N == 0:
            raise IndexError("edge_index out of range: edges on a graph without nodes")
        nat.check(L.mgn_topology_build_async(
            nat.ptr(ei), E, N, nat.ptr(self.csc_src), nat.ptr(self.csc_dst), nat.ptr(self.csc_eid),
            nat.ptr(self.col_ptr), nat.ptr(self.row_ptr), nat.ptr(self.row_perm), nat.ptr(ws), wsb, ew.ptr(),
            nat.stream_ptr(dev)))
        ew.arm()
        self.struct = nat.Topology(N, E, self.csc_src.data_ptr(), self.csc_dst.data_ptr(),
                                   self.csc_eid.data_ptr(), self.col_ptr.data_ptr(),
                                   self.row_ptr.data_ptr(), self.row_perm.data_ptr())


# the block backward's weight-gradient halves run on a side stream, overlapped with the next block's
# data half (set False to serialise them on the current stream, e.g. for A/B timing; same results)
OVERLAP_WGRAD = os.environ.get("MGN_OVERLAP_WGRAD", "0") == "1"
# Gradient-ready callback (data parallelism): EncodeProcessDecode's backward calls
# GRAD_READY(G, lo, hi) on the current stream as soon as the flat-gradient range [lo, hi) is final —
# the decoder's, then each processor block's (last block first), then the encoders' — so a
# bucketed all-reduce can start while the earlier blocks' backward still runs
# (graphphysics.training.distributed.GradBuckets). None: no callbacks.
GRAD_READY = None


def _grad_ready(G, lo, hi):
    if GRAD_READY is not None and hi > lo:
        GRAD_READY(G, lo, hi)


# processor blocks hand the next block's node projections over from their node-MLP kernel
# (mgn_block_forward_chain); False: every block launches its own projection kernel (tests compare)
CHAIN_PROJ = True
# chained bf16 h=128 processor blocks in training: the edge MLP's hidden-layer inputs are not saved by
# the forward; the backward's weight gradients recompute them from e and the block's node projections,
# which stay in a per-block forward workspace (mgn_block_saved.proj, ABI v16; bit-identical inputs, the
# weight-gradient sums in another order). MGN_REW: "auto" (default) for graphs of at least
# REW_MIN_EDGES edges, "1" always, "0" never. Measured (profiles/r05_rew_ab.txt): the saves of a
# cylinder batch-8 block (95k edges, 73 MB) stay in the 256 MB Infinity Cache and cost the forward
# 6 µs, less than the recomputation (-8 % steps/s with it); an aneurysm block's (1.4M edges, 1.1 GB)
# go to HBM and cost 230 µs (+6.6 % steps/s with it)
REW = os.environ.get("MGN_REW", "auto")
REW_MIN_EDGES = 1 << 18
# processor blocks' weight-gradient reductions deferred to one launch after the last block
# (mgn_block_backward_deferred + mgn_wgrad_reduce_many); False: one reduction per block (same sums)
DEFER_REDUCE = True
# data-parallel backward: processor blocks reduced (and handed to GRAD_READY) in groups of about this
# many gradient bytes — one reduction launch per all-reduce bucket instead of one per block
GRAD_GROUP_BYTES = 4 << 20
# deferred path: de / dx handed between consecutive blocks in the pair layout
# (mgn_block_backward_deferred2; bit-identical gradients). MGN_PAIR_DE=0: row-major (A/B timing)
PAIR_DE = os.environ.get("MGN_PAIR_DE", "1") == "1"
# Processor backward with each block's weight-gradient launch on a side stream, beside the next
# block's data-gradient kernels (mgn_block_backward_deferred2 MGN_BWD_DATA_ONLY / _WGRAD_ONLY, two
# workspaces), each on its own share of the CUs (per-call mgn_call_opts caps, ABI v17). MGN_CONC_WGRAD: "auto" (default:
# conc_caps below), "0" (one stream), or "data_cus,wgrad_cus" (0,0: both streams uncapped).
CONC_WGRAD = os.environ.get("MGN_CONC_WGRAD", "auto")
# concurrent backward: workspaces rotated between blocks (MGN_CONC_WS = count or "all" = one per block).
# The data half of block b waits for the weight gradients of block b + count before reusing a workspace,
# which keeps the two streams in lock-step: the ring then reads each block's dZ saves right after they
# were written, from the Infinity Cache (measured: "all" lets the data half run ahead, the saves are
# evicted before the ring reads them and the step slows 337 -> 311 steps/s)
CONC_WS = os.environ.get("MGN_CONC_WS", "2")
# concurrent backward: each block's slab reduction on the side stream right after its weight-gradient
# launch instead of in the one reduction launch at the end of the backward (same sums; measured Cfg B
# 344.1 -> 345.1 steps/s, sustained 352.3 -> 354.6: the end-of-backward reduction leaves the critical
# path). MGN_SIDE_REDUCE=0: one reduction at the end
SIDE_REDUCE = os.environ.get("MGN_SIDE_REDUCE", "1") == "1"
# concurrent backward: the encoders' weight-gradient launches sized for the data share of the CUs
# (MGN_ENC_CAP=0: the weight-gradient share, as the processor's rings)
ENC_DATA_CAP = os.environ.get("MGN_ENC_CAP", "1") == "1"
# concurrent backward: the decoder's weight gradients on the side stream beside the last block's data
# half (MGN_DEC_SPLIT=0: right after its data gradients on the current stream)
DEC_SPLIT = os.environ.get("MGN_DEC_SPLIT", "1") == "1"


def conc_caps(E, chained, dev=None):
    """(data CUs, weight-gradient CUs) of the concurrent backward, or None (one stream). "auto": only
    the chained bf16 h=128 blocks in the latency-bound regime — their persistent edge kernels run 1-4
    16-row tiles per wave on the whole chip (Cfg B: 1.8) — with the chip split 5/8 + 3/8 (MI355X's 256
    CUs: 160 + 96; measured, Cfg B bf16: 332 -> 342 steps/s; 192 + 64: 297, 128 + 128: 322, both
    uncapped: 317). The CU count is the device's (a partitioned device or another SKU scales the split
    and the regime estimate). Measured slower, so one stream: fp32 Cfg B (its MFMA-bound ring: 98 ->
    87), Cfg C at plate.json's sizes (1011 -> 942, uncapped), Cfg E with saved edge inputs (1.4M edges,
    throughput-bound: 33.5 -> 32.7; with the recomputed weight gradients it gains: see below). The small graphs lose to the cross-stream dependencies of the replayed graph even with one
    workspace per block (no wait on the main stream): Cfg A 1720 -> 1515 uncapped / 1420 at 160 + 96,
    Cfg C 1034 -> 870 / 883 (profiles/r04_ab.txt, r04_ab8.sh)."""
    v = CONC_WGRAD
    if v == "0":
        return None
    if v != "auto":
        d, r = (int(t) for t in v.split(","))
        return d, r
    cus = _device_cus(dev)
    tiles_per_wave = E / (16 * 12 * cus)
    if chained and tiles_per_wave > 4.0 and (REW == "1" or (REW == "auto" and E >= REW_MIN_EDGES)):
        # throughput regime with the recomputed weight gradients (Cfg E): the chip split in halves
        # (4 + 4 XCDs), measured 38.4 -> 39.4 steps/s; 160 + 96 and uncapped +1 %, splits off the
        # 32-CU XCD grain (112 + 144, 144 + 112) -11 %, 192 + 64 -19 % (profiles/r05_ab.txt)
        d = cus // 2
        return d, cus - d
    if not (chained and 1.0 <= tiles_per_wave <= 4.0):
        return None
    d = (cus * 5 + 4) // 8
    return d, cus - d


_CUS = {}


def _device_cus(dev):
    """Compute units of the device (MI355X: 256)."""
    dev = torch.device(dev) if dev is not None else torch.device("cuda", torch.cuda.current_device())
    n = _CUS.get(dev.index)
    if n is None:
        n = _CUS[dev.index] = int(torch.cuda.get_device_properties(dev).multi_processor_count)
    return n


_SIDE = {}
# the schedule the last EncodeProcessDecode backward ran (tests assert which path a step took)
LAST_SCHEDULE = {}
# Inspection hook (tests: mask-pinned parity): INSPECT(dict) is called at the end of every training
# forward of EncodeProcessDecode with the forward saves (topology, plan, per-MLP saved buffers), so a
# check can read the ReLU branch each hidden unit took. None: no call.
INSPECT = None


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        s = _SIDE[dev] = torch.cuda.Stream(dev)
    return s


_TOPO_CACHE = []  # [(weakref(edge_index), version, num_nodes, topo)], most recent first
_TOPO_CACHE_MAX = 8


def get_topology(edge_index, num_nodes):
    """Topology for this exact edge_index tensor object (identity + version checked: a freed
    tensor's address reused by a new one never hits a stale entry)."""
    for i, (ref, ver, n, topo) in enumerate(_TOPO_CACHE):
        if ref() is edge_index and ver == edge_index._version and n == num_nodes:
            if i:
                _TOPO_CACHE.insert(0, _TOPO_CACHE.pop(i))
            return topo
    topo = GraphTopology(edge_index, num_nodes)
    _TOPO_CACHE.insert(0, (weakref.ref(edge_index), edge_index._version, num_nodes, topo))
    del _TOPO_CACHE[_TOPO_CACHE_MAX:]
    return topo


def forget_topology(edge_index):
    """Drop the cached topology of this edge_index tensor (its next use rebuilds it, re-validating it
    on the device error word)."""
    _TOPO_CACHE[:] = [ent for ent in _TOPO_CACHE if ent[0]() is not edge_index]


# --------------------------------------------------------------------------- MLPs and plans
KERNEL_WIDTHS = (16, 32, 64, 128, 256)


def kernel_width(h):
    """The hidden width libmgn's kernels run a model of hidden size h on: h itself when the kernels
    are instantiated for it, else the next such width with zero-padded channels (exact: padded
    weights, biases and RMSNorm scales are 0, so every padded channel stays 0 forward and backward,
    and the RMSNorm divides by the true h — mgn_mlp.norm_dim). Above 256: unsupported."""
    for w in KERNEL_WIDTHS:
        if h <= w:
            return w
    raise ValueError(f"hidden_size {h} is not supported by libmgn's kernels (at most {KERNEL_WIDTHS[-1]})")


class MlpSpec:
    """kblocks: layer 0's input is kblocks blocks of `hidden` features ([e ‖ x_i ‖ x_j]: 3, [x ‖ aggr]: 2),
    each padded to the kernel width; 0: a raw input (encoders) whose columns are not padded."""

    def __init__(self, seq, kblocks=0):
        from graphphysics.models.layers import RMSNorm

        mods = list(seq)
        linears = [m for m in mods if isinstance(m, nn.Linear)]
        norm = [m for m in mods if isinstance(m, RMSNorm)]
        expect = []
        for i in range(len(linears)):
            expect.append(nn.Linear)
            if i < len(linears) - 1:
                expect.append(nn.ReLU)
        if norm:
            expect.append(RMSNorm)
        if [type(m) for m in mods] != expect or len(norm) > 1:
            raise ValueError("MLP must be Linear,ReLU,...,Linear[,RMSNorm] (reference build_mlp)")
        if norm and (norm[0].bias or not (norm[0].p < 0.0 or norm[0].p > 1.0) or norm[0].eps != 1e-8):
            raise ValueError("fused RMSNorm supports the reference defaults (p=-1, eps=1e-8, no bias)")
        self.linears = linears
        self.norm = norm[0] if norm else None
        self.n_layers = len(linears)
        self.in_dim = linears[0].in_features
        self.hidden = linears[0].out_features
        self.out_dim = linears[-1].out_features
        self.params = [p for lin in linears for p in (lin.weight, lin.bias)]
        if self.norm is not None:
            self.params.append(self.norm.scale)
        self.numel = sum(p.numel() for p in self.params)
        # kernel geometry (zero-padded when the hidden size is not a kernel width)
        self.width = kernel_width(self.hidden)
        self.padded = self.width != self.hidden
        if kblocks and self.in_dim != kblocks * self.hidden:
            raise ValueError("block MLP input must be %d x hidden" % kblocks)
        self.kblocks = kblocks
        pad_n = lambda n: self.width if n == self.hidden else n  # noqa: E731 (hidden rows padded; the decoder's out not)
        self.shapes = []  # per Linear: (n_pad, k_pad, n, k, kb_src, kb_pad)
        for i, lin in enumerate(linears):
            n, k = lin.out_features, lin.in_features
            if i == 0:
                kp, kbs, kbp = (kblocks * self.width, self.hidden, self.width) if kblocks else (k, 0, 0)
            else:
                kp, kbs, kbp = self.width, self.hidden, self.width
            self.shapes.append((pad_n(n), kp, n, k, kbs, kbp))
        self.out_width = pad_n(self.out_dim)
        # parameter layout of the padded MLP (what the kernels' gradients are written in)
        self.numel_pad = sum(np_ * kp + np_ for np_, kp, *_ in self.shapes) + (self.out_width if self.norm else 0)

    def describe(self, mdt, wpack, wtpack, bias_ptrs=None, scale_ptr=None):
        d = nat.Mlp()
        d.n_layers, d.in_dim, d.hidden, d.out_dim = self.n_layers, self.shapes[0][1], self.width, self.out_width
        d.has_norm, d.dtype = int(self.norm is not None), mdt
        d.norm_dim = self.out_dim if (self.padded and self.norm is not None) else 0
        d.wpack, d.wtpack = wpack, wtpack
        for i, lin in enumerate(self.linears):
            d.bias[i] = bias_ptrs[i] if bias_ptrs is not None else lin.bias.data_ptr()
        if self.norm is not None:
            d.scale = scale_ptr if scale_ptr is not None else self.norm.scale.data_ptr()
        else:
            d.scale = 0
        return d


class _PackedWeights:
    """Fragment-packed copies of all Linear weights of a plan for one (device, dtype); for a plan with
    zero-padded MLPs also the padded fp32 biases / RMSNorm scales the kernels read (refreshed with the
    packs every forward: one gather launch)."""

    def __init__(self, plan, device, mdt):
        L = nat.lib()
        tdt = nat.torch_dtype(mdt)
        regions, jobs, total, max_el = [], [], 0, 1
        for spec in plan.specs:
            per = [int(L.mgn_linear_pack_elems(np_, kp, mdt)) for np_, kp, *_ in spec.shapes]
            regions.append((total, per))
            total += 2 * sum(per)
        self.buf = torch.empty(max(total, 1), dtype=tdt, device=device)
        esz = self.buf.element_size()
        base = self.buf.data_ptr()
        # padded bias / scale vectors: pad_vec[i] = flat_params[pad_idx[i]] (pad_idx -1: 0)
        self.pad_vec = None
        vec_slots = []
        if any(sp.padded for sp in plan.specs):
            vecs, widths = [], []
            for sp in plan.specs:
                if sp.padded:
                    vecs += [lin.bias for lin in sp.linears] + ([sp.norm.scale] if sp.norm is not None else [])
                    widths += [s_[0] for s_ in sp.shapes] + ([sp.out_width] if sp.norm is not None else [])
            # one gather from the parameters' common storage (flatten_parameters: always the case for
            # a flattened model); otherwise (parameters in separate storages) a concatenation
            st0 = vecs[0].untyped_storage()
            self.flat = None
            if all(v.untyped_storage().data_ptr() == st0.data_ptr() for v in vecs):
                self.flat = torch.empty(0, dtype=torch.float32, device=device).set_(st0)
            idx = []
            for v, w in zip(vecs, widths):
                vec_slots.append(len(idx))
                o = v.storage_offset()
                idx += [o + i if i < v.numel() else -1 for i in range(w)]
            pidx = torch.tensor(idx, dtype=torch.int64)
            self.pad_mask = (pidx >= 0).to(device=device, dtype=torch.float32)
            self.pad_idx = pidx.clamp(min=0).to(device)
            self.pad_vec = torch.zeros(len(idx), dtype=torch.float32, device=device)
            self.pad_tmp = torch.zeros_like(self.pad_vec)
            self.vecs, self.widths = vecs, widths
        vbase = self.pad_vec.data_ptr() if self.pad_vec is not None else 0
        slot = iter(vec_slots)
        self.descs = []
        for spec, (off, per) in zip(plan.specs, regions):
            n = sum(per)
            wp, wtp = base + off * esz, base + (off + n) * esz
            o = 0
            for lin, cnt, (np_, kp, n0, k0, kbs, kbp) in zip(spec.linears, per, spec.shapes):
                if spec.padded:
                    j = nat.PackJob(lin.weight.data_ptr(), wp + o * esz, wtp + o * esz, np_, kp, mdt,
                                    n0, k0, kbs if kbp else k0, kbp if kbp else k0, 0)
                else:
                    j = nat.PackJob(lin.weight.data_ptr(), wp + o * esz, wtp + o * esz, np_, kp, mdt, 0, 0, 0, 0, 0)
                jobs.append(j)
                max_el = max(max_el, np_ * kp)
                o += cnt
            if spec.padded:
                bptr = [vbase + 4 * next(slot) for _ in spec.linears]
                sptr = vbase + 4 * next(slot) if spec.norm is not None else None
                self.descs.append(spec.describe(mdt, wp, wtp, bptr, sptr))
            else:
                self.descs.append(spec.describe(mdt, wp, wtp))
        arr = (nat.PackJob * len(jobs))(*jobs)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.jobs = raw.to(device)
        self.njobs, self.max_el = len(jobs), max_el
        self.wptrs = tuple(lin.weight.data_ptr() for s in plan.specs for lin in s.linears)

    def repack(self, stream):
        nat.check(nat.lib().mgn_pack_weights(nat.ptr(self.jobs), self.njobs, self.max_el, stream))
        if self.pad_vec is not None:
            with torch.no_grad():
                if self.flat is not None:
                    torch.index_select(self.flat, 0, self.pad_idx, out=self.pad_tmp)
                    torch.mul(self.pad_tmp, self.pad_mask, out=self.pad_vec)
                else:
                    torch.cat([torch.nn.functional.pad(v.detach().reshape(-1), (0, w - v.numel()))
                               for v, w in zip(self.vecs, self.widths)], out=self.pad_vec)


class ModelPlan:
    """All MLPs of a module, in module.parameters() order. kblocks: per MLP (MlpSpec)."""

    def __init__(self, module, mlps, kblocks=None):
        self.module = module
        self.specs = [MlpSpec(m, kb) for m, kb in zip(mlps, kblocks or [0] * len(mlps))]
        order = [p for s in self.specs for p in s.params]
        mine = list(module.parameters())
        if len(order) != len(mine) or any(a is not b for a, b in zip(order, mine)):
            raise RuntimeError("module parameters are not exactly its MLP parameters in order")
        self.params = mine
        self.offsets = []
        o = 0
        for s in self.specs:
            self.offsets.append(o)
            o += s.numel
        self.numel = o
        # zero-padded MLPs: the kernels write gradients in the padded layout (offsets_pad / numel_pad);
        # unpad_idx gathers the true gradients from it
        self.padded = any(s.padded for s in self.specs)
        self.offsets_pad, self.numel_pad = list(self.offsets), self.numel
        self.unpad_idx = None
        if self.padded:
            self.offsets_pad, idx, o = [], [], 0
            for s in self.specs:
                self.offsets_pad.append(o)
                for lin, (np_, kp, n, k, kbs, kbp) in zip(s.linears, s.shapes):
                    # weight [n][k] inside [np_][kp] (k: blocks of kbs source columns in kbp)
                    c = torch.arange(k)
                    col = (c // kbs) * kbp + c % kbs if kbp else c
                    idx.append((o + torch.arange(n)[:, None] * kp + col[None, :]).reshape(-1))
                    o += np_ * kp
                    idx.append(o + torch.arange(n))  # bias
                    o += np_
                if s.norm is not None:
                    idx.append(o + torch.arange(s.out_dim))
                    o += s.out_width
            self.numel_pad = o
            self._unpad_cpu = torch.cat(idx).to(torch.int64)
            assert self._unpad_cpu.numel() == self.numel
        self._packed = {}

    def unpad(self, Gp):
        """True-layout gradients from the padded layout (one gather)."""
        if self.unpad_idx is None or self.unpad_idx.device != Gp.device:
            self.unpad_idx = self._unpad_cpu.to(Gp.device)
        return torch.index_select(Gp, 0, self.unpad_idx)

    def packed(self, device, mdt):
        key = (str(device), mdt)
        pw = self._packed.get(key)
        wptrs = tuple(lin.weight.data_ptr() for s in self.specs for lin in s.linears)
        if pw is None or pw.wptrs != wptrs:
            pw = _PackedWeights(self, device, mdt)
            self._packed[key] = pw
        return pw

    def grad_views(self, flat):
        out, o = [], 0
        for p in self.params:
            n = p.numel()
            out.append(flat[o:o + n].view_as(p))
            o += n
        return out


def flatten_parameters(module):
    """Re-home every parameter as a view of ONE contiguous fp32 buffer (registration order), so
    the fused optimizer and the gradient all-reduce each see a single buffer."""
    params = list(module.parameters())
    if not params:
        return None
    dev = params[0].device
    if any(p.device != dev or p.dtype != torch.float32 for p in params):
        return None
    flat = torch.empty(sum(p.numel() for p in params), dtype=torch.float32, device=dev)
    o = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            flat[o:o + n].copy_(p.reshape(-1))
            p.data = flat[o:o + n].view_as(p)
            o += n
    module._flat_params = flat
    return flat


# --------------------------------------------------------------------------- helpers
def _empty(n, dtype, device):
    return torch.empty(max(int(n), 1), dtype=dtype, device=device)


def _alloc_mlp_saved(desc, spec, rows, tdt, device, need_z, block_mlp=False, with_act=True):
    """with_act False: the R8 layer inputs are never written (the recomputed edge weight gradients) — a
    one-element placeholder (non-NULL: the training forward's kernels) instead of the full buffer."""
    ae, mw = ctypes.c_int64(), ctypes.c_int64()
    nat.check(nat.lib().mgn_mlp_saved_elems(ctypes.byref(desc), rows, int(block_mlp), ctypes.byref(ae),
                                            ctypes.byref(mw)))
    act = _empty(ae.value if with_act else 1, tdt, device)
    mask = _empty(mw.value, torch.int64, device)
    z = _empty(rows * spec.width, tdt, device) if need_z else None
    rden = _empty(rows, torch.float32, device) if need_z else None
    s = nat.MlpSaved(act.data_ptr(), mask.data_ptr(), z.data_ptr() if z is not None else 0,
                     rden.data_ptr() if rden is not None else 0)
    return s, (act, mask, z, rden)


def _alloc_block_saved(edesc, ndesc, espec, nspec, topo, tdt, device, edge_act=True):
    """edge_act False (mgn_block_saved.proj): the edge MLP's R8 inputs are never written — a
    one-element placeholder (non-NULL: the training forward's kernels)."""
    se, ke = _alloc_mlp_saved(edesc, espec, topo.num_edges, tdt, device, True, True, with_act=edge_act)
    sn, kn = _alloc_mlp_saved(ndesc, nspec, topo.num_nodes, tdt, device, nspec.norm is not None, True)
    aggr = _empty(topo.num_nodes * espec.width, tdt, device)
    return nat.BlockSaved(se, sn, aggr.data_ptr()), (ke, kn, aggr)


def _alloc_block_infer(espec, topo, tdt, device):
    """Inference scratch of mgn_block_forward (act = NULL): the edge MLP's z/rden only."""
    z = _empty(topo.num_edges * espec.width, tdt, device)
    rden = _empty(topo.num_edges, torch.float32, device)
    se = nat.MlpSaved(0, 0, z.data_ptr(), rden.data_ptr())
    return nat.BlockSaved(se, nat.MlpSaved(0, 0, 0, 0), 0), (z, rden)


def _padc(t, H):
    """Columns zero-padded to the kernel width H (no copy when already H wide)."""
    return t if t.shape[1] == H else torch.nn.functional.pad(t, (0, H - t.shape[1]))


def _permute(src, idx, rows, cols, in_mdt, out_tdt, scatter, stream, out=None):
    if out is None:
        out = torch.empty((rows, cols), dtype=out_tdt, device=src.device)
    nat.check(nat.lib().mgn_permute_rows(nat.ptr(src), nat.ptr(out), nat.ptr(idx), rows, cols, in_mdt,
                                         nat.mgn_dtype(out_tdt), int(scatter), stream))
    return out


def _mlp_fwd(desc, spec, inp, in_mdt, in_ld, rows_idx, rows, out, out_mdt, saved, stream):
    nat.check(nat.lib().mgn_mlp_forward(ctypes.byref(desc), nat.ptr(inp), in_mdt, in_ld,
                                        nat.ptr(rows_idx), rows, nat.ptr(out), out_mdt,
                                        ctypes.byref(saved), stream))


def _mlp_bwd(desc, inp, in_mdt, in_ld, rows_idx, rows, saved, dout, dout_mdt, din, din_mdt, grads, ws,
             stream):
    nat.check(nat.lib().mgn_mlp_backward(
        ctypes.byref(desc), nat.ptr(inp), in_mdt, in_ld, nat.ptr(rows_idx), rows, ctypes.byref(saved),
        nat.ptr(dout), dout_mdt, nat.ptr(din), din_mdt, nat.ptr(grads), nat.ptr(ws),
        ws.numel() if ws is not None else 0, stream))


def _mlp_bwd_deferred(desc, inp, in_mdt, in_ld, rows_idx, rows, saved, dout, dout_mdt, din, din_mdt, grads, ws,
                      keep, red, stream, opts=None):
    """_mlp_bwd with the reduction left to one mgn_wgrad_reduce_many at the end of the backward; opts: the
    call's mgn_call_opts (CU caps, error word; ABI v17)."""
    _mlp_bwd_half(desc, inp, in_mdt, in_ld, rows_idx, rows, saved, dout, dout_mdt, din, din_mdt, grads, ws, keep,
                  red, 0, stream, opts)


def _mlp_bwd_half(desc, inp, in_mdt, in_ld, rows_idx, rows, saved, dout, dout_mdt, din, din_mdt, grads, ws, keep,
                  red, flags, stream, opts=None):
    """One half of _mlp_bwd_deferred (mgn_mlp_backward_deferred3, ABI v17): flags MGN_BWD_DATA_ONLY, then
    MGN_BWD_WGRAD_ONLY with the same arguments (red carries the partial-row count between them); 0: whole."""
    nat.check(nat.lib().mgn_mlp_backward_deferred3(
        ctypes.byref(desc), nat.ptr(inp), in_mdt, in_ld, nat.ptr(rows_idx), rows, ctypes.byref(saved),
        nat.ptr(dout), dout_mdt, nat.ptr(din), din_mdt, nat.ptr(grads), nat.ptr(ws), ws.numel(), nat.ptr(keep),
        keep.numel(), red, flags, ctypes.byref(opts) if opts is not None else None, stream))


def _mlp_keep(desc, rows, dev):
    n = int(nat.lib().mgn_mlp_backward_keep_bytes(ctypes.byref(desc), rows))
    return torch.empty(max(n, 256), dtype=torch.uint8, device=dev)


def _ws_bytes_mlp(desc, rows):
    return int(nat.lib().mgn_mlp_backward_workspace_bytes(ctypes.byref(desc), rows))


def _ws_bytes_block(topo, de, dn):
    return int(nat.lib().mgn_block_backward_workspace_bytes(ctypes.byref(topo.struct),
                                                            ctypes.byref(de), ctypes.byref(dn)))


def bspecs_numel(plan, only_processor, i):
    """Parameter count of processor spec i (block b: edge MLP 2b, node MLP 2b + 1)."""
    return plan.specs[i if only_processor else 3 + i].numel


def _fwd_ws_block(topo, de, dn, dev):
    """Scratch for mgn_block_forward (node projections of the edge MLP's layer 0)."""
    n = int(nat.lib().mgn_block_forward_workspace_bytes(ctypes.byref(topo.struct), ctypes.byref(de),
                                                        ctypes.byref(dn)))
    return torch.empty(max(n, 1), dtype=torch.uint8, device=dev)


# --------------------------------------------------------------------------- EncodeProcessDecode
class EPDFunction(torch.autograd.Function):
    """y = EncodeProcessDecode(graph) with the whole processor on libmgn.
    Encoders: specs[0] (nodes), specs[1] (edges); decoder specs[2]; blocks: specs[3+2b],
    specs[4+2b]. only_processor: specs are the blocks only."""

    @staticmethod
    def forward(ctx, plan, mdt, only_processor, grad_mode, x, edge_attr, topo, *params):
        dev = x.device
        st = nat.stream_ptr(dev)
        tdt = nat.torch_dtype(mdt)
        pw = plan.packed(dev, mdt)
        pw.repack(st)
        descs = pw.descs
        N, E = topo.num_nodes, topo.num_edges
        # grad_mode: torch.is_grad_enabled() at the call (a Function's forward runs with grad disabled, and
        # needs_input_grad reports the inputs' requires_grad even under torch.no_grad): no autograd
        # graph -> inference (the chained bf16 blocks run mgn_block_forward's kernels without saves)
        train = grad_mode and any(ctx.needs_input_grad)
        if only_processor:
            bspecs, bdescs = plan.specs, descs
            H = bspecs[0].width  # the kernels' width (zero-padded when != hidden_size)
            x0 = _padc(x.detach(), H).to(tdt).contiguous()
            e0 = _permute(_padc(edge_attr.detach().float(), H).contiguous(), topo.csc_eid, E, H, nat.MGN_F32, tdt,
                          False, st)
            sv_ne = sv_ee = sv_dec = None
            xin = ein = None
        else:
            bspecs, bdescs = plan.specs[3:], descs[3:]
            ne, ee, dec = plan.specs[:3]
            H = ne.width
            xin = x.detach().float().contiguous()
            ein = edge_attr.detach().float().contiguous()
            x0 = torch.empty((N, H), dtype=tdt, device=dev)
            e0 = torch.empty((E, H), dtype=tdt, device=dev)
            sv_ne = _alloc_mlp_saved(descs[0], ne, N, tdt, dev, ne.norm is not None)
            sv_ee = _alloc_mlp_saved(descs[1], ee, E, tdt, dev, ee.norm is not None)
            _mlp_fwd(descs[0], ne, xin, nat.MGN_F32, ne.in_dim, None, N, x0, mdt, sv_ne[0], st)
            _mlp_fwd(descs[1], ee, ein, nat.MGN_F32, ee.in_dim, topo.csc_eid, E, e0, mdt, sv_ee[0], st)
        xs, es, svs = [x0], [e0], []
        nb = len(bspecs) // 2
        scratch = None
        # node projections hand-off: block b's node kernel writes block b+1's P into the other of two
        # workspaces (mgn_block_forward_chain), so blocks after the first launch no projection kernel.
        # rew: one workspace per block, kept for the backward (mgn_block_saved.proj)
        rew = train and (REW == "1" or (REW == "auto" and E >= REW_MIN_EDGES)) and nb > 0 and N > 0 and E > 0 and all(
            nat.lib().mgn_block_forward_inference_supported(ctypes.byref(bdescs[2 * b]), ctypes.byref(bdescs[2 * b + 1]))
            for b in range(nb))
        fwss = [_fwd_ws_block(topo, bdescs[0], bdescs[1], dev) for _ in range(nb if rew else 2)] if nb else None
        # edge-side aggregation scratch (ABI v17, mgn_block_forward_chain2: graphs of high in-degree), one
        # buffer for every block of the stack (each block's partial rows are dead after its node forward)
        agg_scratch = None
        if train and nb:
            sb = int(nat.lib().mgn_block_forward_scratch_bytes(ctypes.byref(topo.struct), ctypes.byref(bdescs[0]),
                                                               ctypes.byref(bdescs[1])))
            if sb:
                agg_scratch = torch.empty(sb, dtype=torch.uint8, device=dev)
        ready = ctypes.c_int32(0)
        for b in range(nb):
            es_, ns_ = bspecs[2 * b], bspecs[2 * b + 1]
            if train or scratch is None:
                if not train and nat.lib().mgn_block_forward_inference_supported(
                        ctypes.byref(bdescs[2 * b]), ctypes.byref(bdescs[2 * b + 1])):
                    sv = _alloc_block_infer(es_, topo, tdt, dev)  # no backward saves
                else:
                    sv = _alloc_block_saved(bdescs[2 * b], bdescs[2 * b + 1], es_, ns_, topo, tdt, dev,
                                            edge_act=not rew)
                if not train:
                    scratch = sv
            else:
                sv = scratch
            x1 = torch.empty((N, H), dtype=tdt, device=dev)
            e1 = torch.empty((E, H), dtype=tdt, device=dev)
            fws, nws = (fwss[b], fwss[min(b + 1, nb - 1)]) if rew else (fwss[b % 2], fwss[(b + 1) % 2])
            if rew:  # the block's projections stay alive for its backward (ctx.state), outside sv[1]
                sv[0].proj = fws.data_ptr()
            nxt = ctypes.byref(bdescs[2 * b + 2]) if CHAIN_PROJ and b + 1 < nb else None
            proj_ready = ready.value
            nat.check(nat.lib().mgn_block_forward_chain2(
                ctypes.byref(topo.struct), ctypes.byref(bdescs[2 * b]), ctypes.byref(bdescs[2 * b + 1]),
                nat.ptr(xs[-1]), nat.ptr(es[-1]), nat.ptr(x1), nat.ptr(e1), ctypes.byref(sv[0]), nat.ptr(fws),
                fws.numel(), proj_ready, nxt, nat.ptr(nws) if nxt is not None else None, nws.numel(),
                ctypes.byref(ready), nat.ptr(agg_scratch), agg_scratch.numel() if agg_scratch is not None else 0, st))
            if train:
                xs.append(x1)
                es.append(e1)
                svs.append(sv)
            else:
                xs, es = [x1], [e1]
        if only_processor:
            out = xs[-1][:, :bspecs[0].hidden].float().contiguous()
        else:
            out = torch.empty((N, dec.out_width), dtype=torch.float32, device=dev)
            sv_dec = _alloc_mlp_saved(descs[2], dec, N, tdt, dev, dec.norm is not None)
            _mlp_fwd(descs[2], dec, xs[-1], mdt, H, None, N, out, nat.MGN_F32, sv_dec[0], st)
            if dec.out_width != dec.out_dim:  # a decoder whose output width is the (padded) hidden size
                out = out[:, :dec.out_dim].contiguous()
        if train and INSPECT is not None:
            # rew: the edge MLPs' R8 inputs were not saved (sv[1][0][0] is a placeholder)
            INSPECT(dict(topo=topo, plan=plan, mdt=mdt, only_processor=only_processor, svs=svs, sv_ne=sv_ne,
                         sv_ee=sv_ee, sv_dec=sv_dec, rew=rew))
        if train:
            ctx.plan, ctx.mdt, ctx.only_processor, ctx.topo = plan, mdt, only_processor, topo
            ctx.pw = pw
            ctx.state = (xin, ein, xs, es, svs, sv_ne, sv_ee, sv_dec)
            ctx.fwss = fwss if rew else None  # rew: per-block node projections read by the backward
            ctx.H = H
        return out

    @staticmethod
    def backward(ctx, gout):
        plan, mdt, topo, pw = ctx.plan, ctx.mdt, ctx.topo, ctx.pw
        xin, ein, xs, es, svs, sv_ne, sv_ee, sv_dec = ctx.state
        dev = xs[0].device
        st = nat.stream_ptr(dev)
        tdt = nat.torch_dtype(mdt)
        N, E, H = topo.num_nodes, topo.num_edges, ctx.H
        descs = pw.descs
        L = nat.lib()
        # the kernels write gradients in the (zero-)padded parameter layout; a plan of kernel-width
        # MLPs has the true layout (offsets_pad == offsets, no gather at the end)
        G = torch.empty(plan.numel_pad, dtype=torch.float32, device=dev)
        gp = G.data_ptr()
        off = plan.offsets_pad
        # gradient-ready ranges are in the true layout: a padded plan hands over everything at the end
        ready = (lambda *_: None) if plan.padded else _grad_ready
        if ctx.only_processor:
            bdescs, boff = descs, off
        else:
            bdescs, boff = descs[3:], off[3:]
        nb = len(bdescs) // 2
        chained = nb > 0 and all(
            L.mgn_block_forward_inference_supported(ctypes.byref(bdescs[2 * b]), ctypes.byref(bdescs[2 * b + 1]))
            for b in range(nb))
        # Each block: the data half (dx, de) on the current stream; the weight-gradient half on a side
        # stream, overlapped with the next block's data half (two workspaces alternate; a workspace is
        # reused only after the side stream has finished with it). Joined before returning.
        overlap = OVERLAP_WGRAD and nb > 1
        # deferred weight-gradient reductions: each block leaves its slabs in its own keep buffer and
        # ONE launch reduces them all after the last block; with a gradient-ready callback (the
        # data-parallel bucketed all-reduce) one launch per group of blocks whose gradients fill a
        # bucket (GRAD_GROUP_BYTES), handed over as one range as soon as the group's backward ends
        defer = DEFER_REDUCE and not overlap and nb > 0
        # concurrent backward (weight-gradient launches beside the next block's data gradients), with or
        # without a gradient-ready callback: under data parallelism each block's slabs are reduced on the
        # side stream right after its ring and the range is handed over THERE, so the bucketed all-reduce
        # waits for the side stream's work, not for the main stream (GradBuckets records per stream)
        caps = conc_caps(E, chained, dev)
        conc = caps is not None and defer and nb > 1
        side_reduced = conc and (SIDE_REDUCE or GRAD_READY is not None)
        # encoders' and decoder's reductions deferred into the final mgn_wgrad_reduce_many too (one
        # reduction launch per backward). With a gradient-ready callback only on the concurrent
        # backward, where the decoder is reduced and handed over right after its weight gradients
        # (early_dec) and the encoders, last anyway, in the final launch
        defer_dense = DEFER_REDUCE and not ctx.only_processor and not OVERLAP_WGRAD and (GRAD_READY is None or conc)
        early_dec = defer_dense and GRAD_READY is not None
        LAST_SCHEDULE.update(conc=caps if conc else None, side_reduced=side_reduced, defer_dense=defer_dense,
                             early_dec=early_dec, grad_ready=GRAD_READY is not None)
        # per-call options (ABI v17): CU caps of the concurrent section's launches, and the device error word
        # the recomputed weight gradients report a hand-off timeout on (the step's AdamW is then skipped and
        # the next poll raises)
        ew = nat.error_word(dev)
        opts0 = nat.CallOpts(0, 0, ew.ptr().value)
        optsc = nat.CallOpts(caps[0], caps[1], ew.ptr().value) if conc else opts0
        optse = nat.CallOpts(caps[0], caps[0] if ENC_DATA_CAP else caps[1], ew.ptr().value) if conc else opts0
        need = _ws_bytes_block(topo, bdescs[0], bdescs[1]) if len(bdescs) >= 2 else 0
        if not ctx.only_processor:
            need = max(need, _ws_bytes_mlp(descs[0], N), _ws_bytes_mlp(descs[1], E),
                       _ws_bytes_mlp(descs[2], N))
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        if defer_dense:
            dreds = (nat.WgradReduce * 3)()  # decoder, node encoder, edge encoder
            keeps = [_mlp_keep(descs[2], N, dev), _mlp_keep(descs[0], N, dev), _mlp_keep(descs[1], E, dev)]
        main = torch.cuda.current_stream(dev)
        side = _side_stream(dev) if (conc or overlap) else None
        dec_args = None

        def dec_wgrad(stream, opts):
            """The decoder's weight-gradient half on `stream` (early_dec: reduced and handed over there)."""
            sp = nat._vp(stream.cuda_stream)
            _mlp_bwd_half(*dec_args, nat.MGN_BWD_WGRAD_ONLY, sp, opts)
            if early_dec:
                nat.check(L.mgn_wgrad_reduce_many(ctypes.pointer(dreds[0]), 1, sp))
                with torch.cuda.stream(stream):
                    ready(G, off[2], off[2] + plan.specs[2].numel)

        if ctx.only_processor:
            dx = _padc(gout.detach(), H).to(tdt).contiguous()
        else:
            dx = torch.empty((N, H), dtype=tdt, device=dev)
            g = _padc(gout.detach().float(), plan.specs[2].out_width).contiguous()
            if defer_dense:
                # the decoder's data gradients now, its weight gradients once the processor's schedule is
                # known (beside the last block's data half on the concurrent backward); own workspace
                wsd = torch.empty(max(_ws_bytes_mlp(descs[2], N), 1), dtype=torch.uint8, device=dev)
                dec_args = (descs[2], xs[-1], mdt, H, None, N, sv_dec[0], g, nat.MGN_F32, dx, mdt,
                            ctypes.c_void_p(gp + 4 * off[2]), wsd, keeps[0], ctypes.pointer(dreds[0]))
                _mlp_bwd_half(*dec_args, nat.MGN_BWD_DATA_ONLY, st, opts0)
                if not (DEC_SPLIT and conc):  # weight gradients at once, on the whole chip
                    dec_wgrad(main, opts0)
                    dec_args = None
            else:
                _mlp_bwd(descs[2], xs[-1], mdt, H, None, N, sv_dec[0], g, nat.MGN_F32, dx, mdt,
                         ctypes.c_void_p(gp + 4 * off[2]), ws, st)
                ready(G, off[2], off[2] + plan.specs[2].numel)
        # the last block's e' is discarded (EncodeProcessDecode returns nodes): its edge-output
        # gradient is zero, which the chained bf16 kernels take as NULL (no zero fill, no reads)
        de = None if nb and nat.lib().mgn_block_forward_inference_supported(
            ctypes.byref(bdescs[2 * nb - 2]), ctypes.byref(bdescs[2 * nb - 1])) else \
            torch.zeros((E, H), dtype=tdt, device=dev)
        pend_hi = pend_b = None  # open group: the range end of its first (highest) block, that block
        # every block on the chained bf16 h=128 kernels (the pair-layout de needs them on both sides;
        # a graph without edges or nodes runs the generic kernels: row-major)
        pair_de = PAIR_DE and not overlap and de is None and N > 0 and E > 0 and chained
        if defer:
            kb = max(int(L.mgn_block_backward_keep_bytes(ctypes.byref(topo.struct), ctypes.byref(bdescs[0]),
                                                         ctypes.byref(bdescs[1]))), 256)
            kb = (kb + 255) // 256 * 256
            keep = torch.empty(nb * kb, dtype=torch.uint8, device=dev)
            reds = (nat.WgradReduce * (2 * nb))()
        if overlap:
            wss = [ws, torch.empty_like(ws)]
            done = [None, None]
        if conc:
            nws = nb if CONC_WS == "all" else max(int(CONC_WS), 2)
            wss = [torch.empty_like(ws) for _ in range(nws)]
            done = [None] * nws
        if dec_args is not None:  # the decoder's weight gradients on the side stream, beside block nb-1's
            ev = torch.cuda.Event()  # data half
            ev.record(main)
            side.wait_event(ev)
            dec_wgrad(side, optsc)
        for b in reversed(range(nb)):
            dx1 = torch.empty((N, H), dtype=tdt, device=dev)
            de1 = torch.empty((E, H), dtype=tdt, device=dev)
            args = (ctypes.byref(topo.struct), ctypes.byref(bdescs[2 * b]), ctypes.byref(bdescs[2 * b + 1]),
                    nat.ptr(xs[b]), nat.ptr(es[b]), ctypes.byref(svs[b][0]), nat.ptr(dx), nat.ptr(de),
                    nat.ptr(dx1), nat.ptr(de1), ctypes.c_void_p(gp + 4 * boff[2 * b]),
                    ctypes.c_void_p(gp + 4 * boff[2 * b + 1]))
            blo = boff[2 * b]
            bhi = boff[2 * b + 1] + bspecs_numel(plan, ctx.only_processor, 2 * b + 1)
            # de / dx between consecutive blocks in the pair layout (the chained kernels' gather
            # layout); the first block's stay row-major (the encoders / the caller read them)
            flags = 0
            if pair_de:
                if b + 1 < nb:
                    flags |= nat.MGN_BWD_DE_OUT_PAIR | nat.MGN_BWD_DX_OUT_PAIR
                if b > 0:
                    flags |= nat.MGN_BWD_DE_PAIR | nat.MGN_BWD_DX_PAIR
            if conc:
                w = wss[b % nws]
                if done[b % nws] is not None:
                    main.wait_event(done[b % nws])  # the side stream is done reading this workspace
                kp = ctypes.c_void_p(keep.data_ptr() + b * kb)
                nat.check(L.mgn_block_backward_deferred3(*args, nat.ptr(w), w.numel(), kp, kb,
                                                         ctypes.pointer(reds[2 * b]),
                                                         flags | nat.MGN_BWD_DATA_ONLY, ctypes.byref(optsc), st))
                ev = torch.cuda.Event()
                ev.record(main)
                side.wait_event(ev)
                sp = nat._vp(side.cuda_stream)
                nat.check(L.mgn_block_backward_deferred3(*args, nat.ptr(w), w.numel(), kp, kb,
                                                         ctypes.pointer(reds[2 * b]),
                                                         flags | nat.MGN_BWD_WGRAD_ONLY, ctypes.byref(optsc), sp))
                if side_reduced:
                    nat.check(L.mgn_wgrad_reduce_many(ctypes.pointer(reds[2 * b]), 2, sp))
                    if GRAD_READY is not None:  # final on the side stream: the bucket waits there
                        with torch.cuda.stream(side):
                            ready(G, blo, bhi)
                ev = torch.cuda.Event()
                ev.record(side)
                done[b % nws] = ev
            elif defer:
                nat.check(L.mgn_block_backward_deferred3(*args, nat.ptr(ws), ws.numel(),
                                                         ctypes.c_void_p(keep.data_ptr() + b * kb), kb,
                                                         ctypes.pointer(reds[2 * b]), flags, ctypes.byref(opts0), st))
                if GRAD_READY is not None:
                    if pend_hi is None:
                        pend_b, pend_hi = b, bhi
                    if (pend_hi - blo) * 4 >= GRAD_GROUP_BYTES or b == 0:
                        # blocks b..pend_b: consecutive descriptors from reds[2b] (a pointer INTO reds)
                        nat.check(L.mgn_wgrad_reduce_many(ctypes.pointer(reds[2 * b]), 2 * (pend_b - b + 1),
                                                          st))
                        ready(G, blo, pend_hi)
                        pend_hi = pend_b = None
            elif not overlap:
                if flags:  # reduced at once (keep = NULL), with the pair-layout hand-offs
                    red2 = (nat.WgradReduce * 2)()
                    nat.check(L.mgn_block_backward_deferred3(*args, nat.ptr(ws), ws.numel(), None, 0, red2,
                                                             flags, ctypes.byref(opts0), st))
                else:
                    nat.check(L.mgn_block_backward(*args, nat.ptr(ws), ws.numel(), st))
                ready(G, blo, bhi)
            else:
                w = wss[b % 2]
                if done[b % 2] is not None:
                    main.wait_event(done[b % 2])  # the side stream is done reading this workspace
                nat.check(L.mgn_block_backward_data(*args, nat.ptr(w), w.numel(), st))
                evd = torch.cuda.Event()
                evd.record(main)
                side.wait_event(evd)
                nat.check(L.mgn_block_backward_wgrad(*args, nat.ptr(w), w.numel(), nat._vp(side.cuda_stream)))
                ev = torch.cuda.Event()
                ev.record(side)
                done[b % 2] = ev
                with torch.cuda.stream(side):
                    ready(G, blo, bhi)
            dx, de = dx1, de1
        # the encoders' backward runs beside block 0's ring launch: with ENC_DATA_CAP its weight-gradient
        # launches take the data share of the chip too (optse; capped at the ring's share they took 63
        # instead of ~40 us)

        def join():  # the side stream's weight gradients are complete before their reduction
            if conc:
                for ev in done:
                    if ev is not None:
                        main.wait_event(ev)

        if defer and not defer_dense and (GRAD_READY is None or conc):
            join()
            if not side_reduced:
                nat.check(L.mgn_wgrad_reduce_many(reds, 2 * nb, st))
        if overlap:
            for ev in done:
                if ev is not None:
                    main.wait_event(ev)  # gradients complete (and both workspaces free) on the main stream
        gx = gea = None
        nx, nea = ctx.needs_input_grad[4], ctx.needs_input_grad[5]
        if ctx.only_processor:
            h = plan.specs[0].hidden
            if nx:
                gx = dx[:, :h].float().contiguous()
            if nea:
                gea = _permute(de, topo.csc_eid, E, H, mdt, torch.float32, True, st)[:, :h].contiguous()
        else:
            ne, ee = plan.specs[0], plan.specs[1]
            gxc = torch.empty((N, ne.in_dim), dtype=torch.float32, device=dev) if nx else None
            gec = torch.empty((E, ee.in_dim), dtype=torch.float32, device=dev) if nea else None
            if defer_dense:
                _mlp_bwd_deferred(descs[0], xin, nat.MGN_F32, ne.in_dim, None, N, sv_ne[0], dx, mdt, gxc,
                                  nat.MGN_F32, ctypes.c_void_p(gp + 4 * off[0]), ws, keeps[1],
                                  ctypes.pointer(dreds[1]), st, optse)
                _mlp_bwd_deferred(descs[1], ein, nat.MGN_F32, ee.in_dim, topo.csc_eid, E, sv_ee[0], de, mdt, gec,
                                  nat.MGN_F32, ctypes.c_void_p(gp + 4 * off[1]), ws, keeps[2],
                                  ctypes.pointer(dreds[2]), st, optse)
                join()
                # ONE reduction for the whole model: decoder (unless reduced already), every processor
                # block (unless reduced on the side stream), encoders
                parts = ([] if early_dec else [dreds[0]]) + \
                    ([reds[i] for i in range(2 * nb)] if defer and not side_reduced else []) + [dreds[1], dreds[2]]
                allr = (nat.WgradReduce * len(parts))(*parts)
                nat.check(L.mgn_wgrad_reduce_many(allr, len(allr), st))
            else:
                _mlp_bwd(descs[0], xin, nat.MGN_F32, ne.in_dim, None, N, sv_ne[0], dx, mdt, gxc, nat.MGN_F32,
                         ctypes.c_void_p(gp + 4 * off[0]), ws, st)
                _mlp_bwd(descs[1], ein, nat.MGN_F32, ee.in_dim, topo.csc_eid, E, sv_ee[0], de, mdt, gec,
                         nat.MGN_F32, ctypes.c_void_p(gp + 4 * off[1]), ws, st)
            gx = gxc
            if nea:
                gea = _permute(gec, topo.csc_eid, E, ee.in_dim, nat.MGN_F32, torch.float32, True, st)
            ready(G, off[0], off[1] + plan.specs[1].numel)
        if plan.padded:
            G = plan.unpad(G)
            _grad_ready(G, 0, plan.numel)
        ctx.state = ctx.fwss = None
        return (None, None, None, None, gx, gea, None, *plan.grad_views(G))


# --------------------------------------------------------------------------- GraphNetBlock
class BlockFunction(torch.autograd.Function):
    """(x', e') = GraphNetBlock(x, edge_index, e) with edges in the CALLER's order."""

    @staticmethod
    def forward(ctx, plan, mdt, grad_mode, x, edge_attr, topo, *params):
        dev = x.device
        st = nat.stream_ptr(dev)
        tdt = nat.torch_dtype(mdt)
        pw = plan.packed(dev, mdt)
        pw.repack(st)
        espec, nspec = plan.specs
        h, H = espec.hidden, espec.width  # hidden size, kernel width (zero-padded when they differ)
        N, E = topo.num_nodes, topo.num_edges
        x0 = _padc(x.detach(), H).to(tdt).contiguous()
        ea = edge_attr.detach()
        if ea.dtype not in (torch.float32, torch.bfloat16):  # fp16 (autocast), fp64, ...: read as fp32
            ea = ea.float()
        if ea.dim() != 2 or ea.shape[0] != E or ea.shape[1] != h:
            raise ValueError(f"edge_attr must have shape [{E}, {h}], got {list(ea.shape)}")
        e0 = _permute(_padc(ea, H).contiguous(), topo.csc_eid, E, H, nat.mgn_dtype(ea.dtype), tdt, False, st) \
            if E else torch.empty((0, H), dtype=tdt, device=dev)
        train = grad_mode and any(ctx.needs_input_grad)  # as EPDFunction
        if not train and nat.lib().mgn_block_forward_inference_supported(ctypes.byref(pw.descs[0]),
                                                                         ctypes.byref(pw.descs[1])):
            sv = _alloc_block_infer(espec, topo, tdt, dev)
        else:
            sv = _alloc_block_saved(pw.descs[0], pw.descs[1], espec, nspec, topo, tdt, dev)
        x1 = torch.empty((N, H), dtype=tdt, device=dev)
        e1 = torch.empty((max(E, 1), H), dtype=tdt, device=dev)
        fws = _fwd_ws_block(topo, pw.descs[0], pw.descs[1], dev)
        nat.check(nat.lib().mgn_block_forward(
            ctypes.byref(topo.struct), ctypes.byref(pw.descs[0]), ctypes.byref(pw.descs[1]), nat.ptr(x0),
            nat.ptr(e0), nat.ptr(x1), nat.ptr(e1), ctypes.byref(sv[0]), nat.ptr(fws), fws.numel(), st))
        e_out = _permute(e1, topo.csc_eid, E, H, mdt, x.dtype, True, st) if E else \
            torch.empty((0, H), dtype=x.dtype, device=dev)
        if train:
            ctx.plan, ctx.mdt, ctx.topo, ctx.pw = plan, mdt, topo, pw
            ctx.state = (x0, e0, sv)
            ctx.xdtype = x.dtype
        if H != h:
            return x1[:, :h].to(x.dtype).contiguous(), e_out[:, :h].contiguous()
        return x1.to(x.dtype), e_out

    @staticmethod
    def backward(ctx, gx, ge):
        plan, mdt, topo, pw = ctx.plan, ctx.mdt, ctx.topo, ctx.pw
        x0, e0, sv = ctx.state
        dev = x0.device
        st = nat.stream_ptr(dev)
        tdt = nat.torch_dtype(mdt)
        N, E = topo.num_nodes, topo.num_edges
        h, H = plan.specs[0].hidden, plan.specs[0].width
        dxo = _padc((gx if gx is not None else torch.zeros((N, h), device=dev)).detach(), H).to(tdt).contiguous()
        if ge is None or E == 0:
            deo = torch.zeros((max(E, 1), H), dtype=tdt, device=dev)
        else:
            deo = _permute(_padc(ge.detach().float(), H).contiguous(), topo.csc_eid, E, H, nat.MGN_F32, tdt, False,
                           st)
        G = torch.empty(plan.numel_pad, dtype=torch.float32, device=dev)
        ws = torch.empty(max(_ws_bytes_block(topo, pw.descs[0], pw.descs[1]), 1), dtype=torch.uint8,
                         device=dev)
        dx = torch.empty((N, H), dtype=tdt, device=dev)
        de = torch.empty((max(E, 1), H), dtype=tdt, device=dev)
        nat.check(nat.lib().mgn_block_backward(
            ctypes.byref(topo.struct), ctypes.byref(pw.descs[0]), ctypes.byref(pw.descs[1]), nat.ptr(x0),
            nat.ptr(e0), ctypes.byref(sv[0]), nat.ptr(dxo), nat.ptr(deo), nat.ptr(dx), nat.ptr(de),
            ctypes.c_void_p(G.data_ptr()), ctypes.c_void_p(G.data_ptr() + 4 * plan.offsets_pad[1]),
            nat.ptr(ws), ws.numel(), st))
        gxo = dx[:, :h].to(ctx.xdtype).contiguous() if ctx.needs_input_grad[3] else None
        geo = None
        if ctx.needs_input_grad[4]:
            geo = _permute(de, topo.csc_eid, E, H, mdt, torch.float32, True, st)[:, :h].contiguous() if E else \
                torch.zeros((0, h), device=dev)
        if plan.padded:
            G = plan.unpad(G)
        ctx.state = None
        return (None, None, None, gxo, geo, None, *plan.grad_views(G))
