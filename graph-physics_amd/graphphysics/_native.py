"""ctypes binding of libmgn (include/mgn.h) — the MI355X-native hot path.

The library is built in-tree by `python __graft_entry__.py` (hipcc --offload-arch=gfx950) into
graph-physics_amd/graphphysics/_lib/libmgn.so. There is NO fallback: every model entry point
raises if the library or a HIP device is missing.
"""
import ctypes
import os

import torch

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libmgn.so")
ABI_VERSION = 17  # include/mgn.h MGN_ABI_VERSION these bindings are written for

MGN_F32 = 0
MGN_BF16 = 1
MGN_BWD_DE_OUT_PAIR = 1  # mgn.h: de_out in the pair layout
MGN_BWD_DE_PAIR = 2      # mgn.h: write de in the pair layout
MGN_BWD_DX_OUT_PAIR = 4  # mgn.h: dx_out in the pair layout
MGN_BWD_DX_PAIR = 8      # mgn.h: write dx in the pair layout
MGN_BWD_DATA_ONLY = 16   # mgn.h (v13): the data-gradient half of mgn_block_backward_deferred2
MGN_BWD_WGRAD_ONLY = 32  # mgn.h (v13): its weight-gradient half
MGN_MAX_LAYERS = 8

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t
_dbl = ctypes.c_double
_f32 = ctypes.c_float
_u32 = ctypes.c_uint32


class Topology(ctypes.Structure):
    _fields_ = [("num_nodes", _i64), ("num_edges", _i64), ("csc_src", _vp), ("csc_dst", _vp),
                ("csc_eid", _vp), ("col_ptr", _vp), ("row_ptr", _vp), ("row_perm", _vp)]


class Mlp(ctypes.Structure):
    _fields_ = [("n_layers", _i32), ("in_dim", _i32), ("hidden", _i32), ("out_dim", _i32),
                ("has_norm", _i32), ("dtype", _i32), ("norm_dim", _i32), ("reserved", _i32),
                ("wpack", _vp), ("wtpack", _vp), ("bias", _vp * MGN_MAX_LAYERS), ("scale", _vp)]


class MlpSaved(ctypes.Structure):
    _fields_ = [("act", _vp), ("mask", _vp), ("z", _vp), ("rden", _vp)]


class BlockSaved(ctypes.Structure):
    _fields_ = [("edge", MlpSaved), ("node", MlpSaved), ("aggr", _vp), ("proj", _vp)]


class WgradReduce(ctypes.Structure):
    _fields_ = [("part", _vp), ("dsp", _vp), ("grads", _vp), ("G", _i64), ("nchunks", _i32), ("ntiles", _i32),
                ("NS", _i32), ("blocks", _i32), ("w0_n", _i32), ("w0_k", _i32), ("xcol0", _i32), ("nchunks_x", _i32),
                ("hoff", _i64), ("nchunks_h", _i32), ("pad", _i32)]


class CallOpts(ctypes.Structure):
    """mgn_call_opts (ABI v17): per-call CU caps and the device error word (mgn.h)."""
    _fields_ = [("data_cus", _i32), ("wgrad_cus", _i32), ("err_word", _vp)]


class NormalizerState(ctypes.Structure):
    _fields_ = [("acc_sum", _vp), ("acc_sum_sq", _vp), ("acc_count", _vp), ("num_acc", _vp), ("pending", _vp),
                ("max_acc", _f32), ("eps", _f32)]


class PackJob(ctypes.Structure):
    _fields_ = [("w", _vp), ("dst", _vp), ("dstT", _vp), ("n", _i32), ("k", _i32), ("dtype", _i32),
                ("n_src", _i32), ("k_src", _i32), ("kb_src", _i32), ("kb_pad", _i32), ("reserved", _i32)]


EXPORTS = {
    "mgn_abi_version": (_i32, []),
    "mgn_last_error": (ctypes.c_char_p, []),
    "mgn_topology_workspace_bytes": (_sz, [_i64, _i64]),
    "mgn_topology_build": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgn_topology_build_async": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp, _vp]),
    "mgn_linear_pack_elems": (_i64, [_i32, _i32, _i32]),
    "mgn_mlp_pack_elems": (_i64, [ctypes.POINTER(Mlp)]),
    "mgn_pack_weights": (_i32, [_vp, _i32, _i64, _vp]),
    "mgn_mlp_forward": (_i32, [ctypes.POINTER(Mlp), _vp, _i32, _i64, _vp, _i64, _vp, _i32,
                               ctypes.POINTER(MlpSaved), _vp]),
    "mgn_mlp_backward_workspace_bytes": (_sz, [ctypes.POINTER(Mlp), _i64]),
    "mgn_mlp_saved_elems": (_i32, [ctypes.POINTER(Mlp), _i64, _i32, _vp, _vp]),
    "mgn_mlp_backward": (_i32, [ctypes.POINTER(Mlp), _vp, _i32, _i64, _vp, _i64,
                                ctypes.POINTER(MlpSaved), _vp, _i32, _vp, _i32, _vp, _vp, _sz, _vp]),
    "mgn_mlp_backward_keep_bytes": (_sz, [ctypes.POINTER(Mlp), _i64]),
    "mgn_mlp_backward_deferred": (_i32, [ctypes.POINTER(Mlp), _vp, _i32, _i64, _vp, _i64,
                                         ctypes.POINTER(MlpSaved), _vp, _i32, _vp, _i32, _vp, _vp, _sz, _vp, _sz,
                                         ctypes.POINTER(WgradReduce), _vp]),
    "mgn_mlp_backward_deferred2": (_i32, [ctypes.POINTER(Mlp), _vp, _i32, _i64, _vp, _i64,
                                          ctypes.POINTER(MlpSaved), _vp, _i32, _vp, _i32, _vp, _vp, _sz, _vp, _sz,
                                          ctypes.POINTER(WgradReduce), _i32, _vp]),
    "mgn_block_forward_inference_supported": (_i32, [ctypes.POINTER(Mlp), ctypes.POINTER(Mlp)]),
    "mgn_block_forward_workspace_bytes": (_sz, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp),
                                                ctypes.POINTER(Mlp)]),
    "mgn_block_forward": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                 _vp, _vp, _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _sz, _vp]),
    "mgn_block_forward_chain": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                       _vp, _vp, _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _sz, _i32,
                                       ctypes.POINTER(Mlp), _vp, _sz, ctypes.POINTER(ctypes.c_int32), _vp]),
    "mgn_block_forward_scratch_bytes": (_sz, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp)]),
    "mgn_block_forward_chain2": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                        _vp, _vp, _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _sz, _i32,
                                        ctypes.POINTER(Mlp), _vp, _sz, ctypes.POINTER(ctypes.c_int32), _vp, _sz, _vp]),
    "mgn_block_backward_workspace_bytes": (_sz, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp),
                                                 ctypes.POINTER(Mlp)]),
    "mgn_block_backward": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                  _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _vp, _vp, _vp, _vp, _vp,
                                  _vp, _sz, _vp]),
    "mgn_block_backward_data": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                       _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _sz, _vp]),
    "mgn_block_backward_wgrad": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                        _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _vp, _vp, _vp, _vp, _vp,
                                        _vp, _sz, _vp]),
    "mgn_block_backward_keep_bytes": (_sz, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp)]),
    "mgn_block_backward_deferred": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                           _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _vp, _vp, _vp, _vp, _vp,
                                           _vp, _sz, _vp, _sz, ctypes.POINTER(WgradReduce), _vp]),
    "mgn_block_backward_deferred2": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                            _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _sz, _vp, _sz, ctypes.POINTER(WgradReduce), _i32, _vp]),
    "mgn_wgrad_reduce_many": (_i32, [ctypes.POINTER(WgradReduce), _i32, _vp]),
    "mgn_block_backward_deferred3": (_i32, [ctypes.POINTER(Topology), ctypes.POINTER(Mlp), ctypes.POINTER(Mlp),
                                            _vp, _vp, ctypes.POINTER(BlockSaved), _vp, _vp, _vp, _vp, _vp, _vp,
                                            _vp, _sz, _vp, _sz, ctypes.POINTER(WgradReduce), _i32,
                                            ctypes.POINTER(CallOpts), _vp]),
    "mgn_mlp_backward_deferred3": (_i32, [ctypes.POINTER(Mlp), _vp, _i32, _i64, _vp, _i64,
                                          ctypes.POINTER(MlpSaved), _vp, _i32, _vp, _i32, _vp, _vp, _sz, _vp, _sz,
                                          ctypes.POINTER(WgradReduce), _i32, ctypes.POINTER(CallOpts), _vp]),
    "mgn_debug_wave_times": (_i32, [_i32, _vp, _i32]),
    "mgn_permute_rows": (_i32, [_vp, _vp, _vp, _i64, _i32, _i32, _i32, _i32, _vp]),
    "mgn_segment_sum": (_i32, [_vp, _vp, _i64, _i32, _i32, _vp, _vp]),
    "mgn_column_stats_workspace_bytes": (_sz, [_i64, _i32]),
    "mgn_column_stats": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp, _sz, _vp]),
    "mgn_normalizer_workspace_bytes": (_sz, [_i64, _i32]),
    "mgn_normalizer_forward": (_i32, [_vp, _i64, _i32, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _vp,
                                      _vp, _sz, _vp]),
    "mgn_simulator_preamble_workspace_bytes": (_sz, [_i64, _i64]),
    "mgn_simulator_preamble": (_i32, [_vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64,
                                      _i32, _i64, _i32, ctypes.POINTER(NormalizerState),
                                      ctypes.POINTER(NormalizerState), ctypes.POINTER(NormalizerState), _vp, _vp,
                                      _vp, _vp, _vp, _sz, _vp]),
    "mgn_simulator_statistics": (_i32, [_vp, _i64, _i64, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp, _i64,
                                        _i32, _i64, _vp, _vp, _vp, _sz, _vp]),
    "mgn_masked_mse_workspace_bytes": (_sz, [_i64]),
    "mgn_masked_mse": (_i32, [_vp, _vp, _i64, _i32, _vp, _i64, _u32, _vp, _vp, _vp, _vp, _sz, _vp]),
    "mgn_masked_mse_backward": (_i32, [_vp, _vp, _i64, _i32, _vp, _i64, _u32, _vp, _vp, _vp, _vp]),
    "mgn_adamw": (_i32, [_vp, _vp, _vp, _vp, _i64, _dbl, _dbl, _dbl, _dbl, _dbl, _i64, _vp]),
    "mgn_adamw_dev": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _dbl, _dbl, _dbl, _dbl, _vp, _vp]),
    "mgn_adamw_dev2": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _dbl, _dbl, _dbl, _dbl, _vp, _i32, _vp]),
    "mgn_coalesce_workspace_bytes": (_sz, [_i64]),
    "mgn_coalesce": (_i32, [_vp, _i64, _i64, _i32, _vp, _vp, _vp, _sz, _vp]),
    "mgn_face_to_edge_keys": (_i64, [_i32, _i64]),
    "mgn_face_to_edge": (_i32, [_vp, _i32, _i64, _i64, _vp, _vp, _vp, _sz, _vp]),
    "mgn_khop_count_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "mgn_khop_count": (_i32, [_vp, _i64, _vp, _i64, _i64, _vp, _vp, _sz, _vp]),
    "mgn_khop_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "mgn_khop_hop": (_i32, [_vp, _i64, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _sz, _vp]),
    "mgn_edge_features": (_i32, [_vp, _i64, _i32, _vp, _i64, _i64, _vp, _i64, _vp, _sz, _vp]),
    "mgn_radius_pairs_workspace_bytes": (_sz, [_i64]),
    "mgn_radius_pairs": (_i32, [_vp, _i64, _i32, _i64, _dbl, _vp, _i64, _vp, _i64, _vp, _vp, _sz, _vp]),
    "mgn_profile_enable": (_i32, [_i32]),
    "mgn_profile_collect": (_i32, [_i32, _vp, _vp]),
}

PROF_KINDS = ["fwd_edge", "fwd_node", "fwd_dense", "bwd_edge", "bwd_node", "bwd_dense", "wgrad",
              "wgrad_reduce", "combine", "pack", "adamw", "proj", "wgrad_dense"]


def profile_enable(on=True):
    check(lib().mgn_profile_enable(int(on)))


def profile_collect():
    """{kernel class: (total_ms, launches)} since the last profile_enable()."""
    out = {}
    for i, name in enumerate(PROF_KINDS):
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        check(lib().mgn_profile_collect(i, ctypes.byref(ms), ctypes.byref(cnt)))
        out[name] = (ms.value, cnt.value)
    return out

_lib = None


def load(path=LIB_PATH):
    """Load libmgn and bind every exported symbol (no device needed)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libmgn not built ({path} missing): run `python __graft_entry__.py` (hipcc gfx950). "
            "The MGN path has no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mgn_abi_version() != ABI_VERSION:  # a stale build would mis-read changed signatures
        raise RuntimeError(f"libmgn ABI {lib.mgn_abi_version()} at {path}, these bindings need {ABI_VERSION}: "
                           "rebuild (python __graft_entry__.py)")
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def check(rc):
    if rc != 0:
        msg = lib().mgn_last_error().decode(errors="replace")
        if "out of range" in msg:
            raise IndexError(msg)
        raise RuntimeError(f"libmgn error {rc}: {msg}")


# ---------------------------------------------------------------- device error word (ABI v7)
ERR_EDGE_INDEX, ERR_TYPE_NEG, ERR_TYPE_BIG = 1, 2, 4
ERR_HANDOFF = 8  # ABI v17: a pipelined kernel's bounded hand-off wait timed out (mgn.h MGN_ERR_HANDOFF)
ERR_ANY, ERR_SKIP_SHIFT, ERR_STALE = 0xFFFF, 16, 1 << 31  # ABI v11 (include/mgn.h)


def _raise_for(bits):
    """The exception the reference raises for the validation failure in `bits`. The exception's
    `mgn_skipped_updates` is the number of optimizer steps mgn_adamw_dev skipped because the error
    was pending (the caller rewinds its host-side step counters by as many)."""
    ex = None
    if bits & ERR_EDGE_INDEX:
        ex = IndexError("edge_index out of range: an index is outside [0, num_nodes) "
                        "(libmgn device check; the reference's ATen gather raises IndexError)")
    elif bits & ERR_TYPE_NEG:
        ex = RuntimeError("Class values must be non-negative.")  # F.one_hot (reference simulator one-hot)
    elif bits & ERR_TYPE_BIG:
        ex = RuntimeError("Class values must be smaller than num_classes.")
    elif bits & ERR_HANDOFF:
        # not a validation error of the batch: a libmgn kernel (the recomputed edge weight gradients)
        # gave up waiting inside its pipeline and wrote NaN partial sums; the optimizer step was skipped
        ex = RuntimeError("libmgn: a hand-off wait of the recomputed weight gradients timed out "
                          "(MGN_ERR_HANDOFF); the step's gradients are invalid and its optimizer update was skipped")
    if ex is not None:
        ex.mgn_skipped_updates = (bits >> ERR_SKIP_SHIFT) & 0xFF
        raise ex


class ErrorWord:
    """One uint32 device word per device that libmgn's validating kernels OR MGN_ERR_* bits into
    (mgn_topology_build_async, mgn_simulator_preamble / _statistics), so a new batch never forces a
    host read-back. arm() queues a non-blocking copy to pinned host memory behind the launches;
    poll() raises (and clears the word) once a queued copy has landed with a bit set — at most one
    call late, without synchronising; check() synchronises and raises now."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.dev = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.event = None

    def ptr(self):
        return _vp(self.dev.data_ptr())

    def arm(self):
        """Queue the device word's copy-back (skipped while a hipGraph is being captured: a captured
        step's owner arms after each replay)."""
        if torch.cuda.is_current_stream_capturing():
            return
        self.host.copy_(self.dev, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.event = ev

    def poll(self):
        ev = self.event
        if ev is None or torch.cuda.is_current_stream_capturing() or not ev.query():
            return
        self.event = None
        bits = int(self.host[0])
        if bits:
            self._clear()
            _raise_for(bits)

    def check(self):
        if torch.cuda.is_current_stream_capturing():
            return
        torch.cuda.current_stream(self.device).synchronize()
        bits = int(self.dev[0].item())
        self.event = None
        if bits:
            self._clear()
            _raise_for(bits)

    def _clear(self):
        self.dev.zero_()
        self.host.zero_()


_ERR_WORDS = {}


def error_word(device):
    d = torch.device(device)
    if d.index is None:
        d = torch.device(d.type, torch.cuda.current_device())
    w = _ERR_WORDS.get(d)
    if w is None:
        if torch.cuda.is_current_stream_capturing():  # its storage must outlive any graph pool
            raise RuntimeError("libmgn: run one eager call on this device before capturing a graph")
        w = _ERR_WORDS[d] = ErrorWord(d)
    return w


def poll_errors(device=None):
    """Raise a validation error some earlier libmgn launch flagged, if its copy-back has landed."""
    for d, w in list(_ERR_WORDS.items()):
        if device is None or torch.device(device) == d or torch.device(device).index is None:
            w.poll()


def check_errors(device=None):
    """Synchronise and raise any validation error libmgn flagged on the device word(s)."""
    for d, w in list(_ERR_WORDS.items()):
        if device is None or torch.device(device) == d or torch.device(device).index is None:
            w.check()


def require_device(t):
    if not t.is_cuda:
        raise RuntimeError("the MI355X MGN path needs tensors on a HIP device (no CPU fallback)")


def stream_ptr(device=None):
    return _vp(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    """Device address of a tensor (None -> NULL; raw ints / c_void_p pass through)."""
    if t is None:
        return _vp(0)
    if isinstance(t, _vp):
        return t
    if isinstance(t, int):
        return _vp(t)
    return _vp(t.data_ptr())


def mgn_dtype(torch_dtype):
    if torch_dtype == torch.float32:
        return MGN_F32
    if torch_dtype == torch.bfloat16:
        return MGN_BF16
    raise ValueError(f"unsupported compute dtype {torch_dtype}")


def torch_dtype(mdt):
    return torch.float32 if mdt == MGN_F32 else torch.bfloat16


def column_stats(x):
    """(Σ_rows x, Σ_rows x²) of a 2-D fp32 HIP tensor as two [1, cols] tensors (mgn_column_stats)."""
    import torch

    require_device(x)
    if x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1:
        x = x.float().contiguous()
    rows, cols = x.shape
    out = torch.empty(2 * cols, dtype=torch.float32, device=x.device)
    ws = torch.empty(max(int(lib().mgn_column_stats_workspace_bytes(rows, cols)), 4), dtype=torch.uint8,
                     device=x.device)
    check(lib().mgn_column_stats(ptr(x), rows, cols, x.stride(0), ptr(out), ptr(ws), ws.numel(),
                                 stream_ptr(x.device)))
    return out[:cols].view(1, cols), out[cols:].view(1, cols)


def normalizer_state(n, accumulate):
    """mgn_normalizer_state of a graphphysics Normalizer module (buffers updated in place)."""
    pend = n._pending_packed if accumulate else None
    return NormalizerState(n._acc_sum.data_ptr(), n._acc_sum_squared.data_ptr(), n._acc_count.data_ptr(),
                           n._num_accumulations.data_ptr(), pend.data_ptr() if pend is not None else None,
                           float(n._max_accumulations), n._eps())


def simulator_preamble(x, y, edge_attr, feat, out, type_index, n_types, accumulate, out_norm, node_norm,
                       edge_norm):
    """Simulator._build_input_graph's three Normalizer.forward calls on libmgn
    (mgn_simulator_preamble): returns (target_normalized [N, out], node_features_normalized
    [N, nf + n_types], edge_attr_normalized [E, de] or None)."""
    import torch

    require_device(x)
    N, E = x.shape[0], (edge_attr.shape[0] if edge_norm is not None else 0)
    dev = x.device
    to = torch.empty((N, out[1] - out[0]), dtype=torch.float32, device=dev)
    no = torch.empty((N, feat[1] - feat[0] + n_types), dtype=torch.float32, device=dev)
    eo = torch.empty((E, edge_attr.shape[1]), dtype=torch.float32, device=dev) if edge_norm is not None else None
    ws = torch.empty(int(lib().mgn_simulator_preamble_workspace_bytes(N, E)), dtype=torch.uint8, device=dev)
    acc = bool(accumulate)
    st = [normalizer_state(n, acc) if n is not None else None for n in (out_norm, node_norm, edge_norm)]
    check(lib().mgn_simulator_preamble(
        ptr(x), N, x.stride(0), feat[0], feat[1], type_index, n_types, out[0], out[1], ptr(y), y.stride(0),
        ptr(edge_attr) if eo is not None else None, E, edge_attr.shape[1] if eo is not None else 0,
        edge_attr.stride(0) if eo is not None else 0, int(acc), ctypes.byref(st[0]), ctypes.byref(st[1]),
        ctypes.byref(st[2]) if st[2] is not None else None, ptr(to), ptr(no), ptr(eo), error_word(dev).ptr(),
        ptr(ws), ws.numel(), stream_ptr(dev)))
    error_word(dev).arm()
    return to, no, eo


def simulator_statistics(x, y, edge_attr, feat, out, type_index, n_types, packed):
    """Batch statistics of the Simulator's three normalizers into `packed` (mgn_simulator_statistics);
    edge_attr None: two normalizers."""
    import torch

    require_device(x)
    N = x.shape[0]
    E = edge_attr.shape[0] if edge_attr is not None else 0
    ws = torch.empty(int(lib().mgn_simulator_preamble_workspace_bytes(N, E)), dtype=torch.uint8, device=x.device)
    check(lib().mgn_simulator_statistics(
        ptr(x), N, x.stride(0), feat[0], feat[1], type_index, n_types, out[0], out[1], ptr(y), y.stride(0),
        ptr(edge_attr), E, edge_attr.shape[1] if edge_attr is not None else 0,
        edge_attr.stride(0) if edge_attr is not None else 0, ptr(packed), error_word(x.device).ptr(), ptr(ws),
        ws.numel(), stream_ptr(x.device)))
    error_word(x.device).arm()
    return packed


def normalizer_forward(x, accumulate, pending, acc_sum, acc_sum_sq, acc_count, num_acc, max_acc, eps):
    """Normalizer.forward on libmgn (mgn_normalizer_forward): updates the fp32 buffers in place when
    accumulating and returns (x - mean) / std as a new contiguous fp32 tensor. pending: None or a
    float32 [2*cols + 1] device tensor {Σx, Σx², count}."""
    import torch

    require_device(x)
    if x.dtype != torch.float32 or x.dim() != 2 or x.stride(1) != 1:
        x = x.float().contiguous()
    rows, cols = x.shape
    out = torch.empty((rows, cols), dtype=torch.float32, device=x.device)
    ws = torch.empty(max(int(lib().mgn_normalizer_workspace_bytes(rows, cols)), 4), dtype=torch.uint8,
                     device=x.device)
    check(lib().mgn_normalizer_forward(ptr(x), rows, cols, x.stride(0), int(bool(accumulate)),
                                       ptr(pending) if pending is not None else None, ptr(acc_sum),
                                       ptr(acc_sum_sq), ptr(acc_count), ptr(num_acc), float(max_acc),
                                       float(eps), ptr(out), ptr(ws), ws.numel(), stream_ptr(x.device)))
    return out
