"""Mask-pinned parity (test infrastructure).

libmgn's forward saves the input of every Linear after the first — the ReLU output of the previous
hidden layer — in the row-octet (R8) layout of include/mgn.h `mgn_mlp_saved` (element (m, c) at
((m/8)·cols + c)·8 + m%8, rows padded to 64; per-layer blocks at mgn_common.h `act_off`). In fp32 a
saved activation is > 0 exactly where the kernel's ReLU passed its pre-activation, so these buffers
give the branch libmgn took for every hidden unit of every MLP. Evaluating the oracle (the reference's
own ops, oracle/mgn_oracle.py) in fp64 on THAT branch (`masks=`) removes the one discontinuity of the
algorithm — a pre-activation within fp32 rounding of 0 that another summation order puts on the other
side of a ReLU — so what remains between libmgn fp32 and the pinned fp64 evaluation is rounding only
(gradients rel-L2 ≤ 1e-3; measured ~1e-6).

Reference: build_mlp layers.py:77-113, GraphNetBlock layers.py:630-746, processors.py:111-137.
"""
import torch


def _rows_pad(m):
    return (m + 63) // 64 * 64


def _rup(a, b):
    return (a + b - 1) // b * b


def _r8(act, off, rows, cols):
    rp = _rows_pad(rows)
    a = act[off:off + rp * cols].view(rp // 8, cols, 8).transpose(1, 2).reshape(rp, cols)
    return a[:rows]


def _mlp_masks(spec, act, rows, gathered, kstep, device="cpu"):
    """[bool [rows, hidden] per hidden layer] of one MLP from its saved act buffer."""
    rp = _rows_pad(rows)
    cols = _rup(spec.width, kstep)
    off = 0 if gathered else rp * _rup(spec.shapes[0][1], kstep)
    out = []
    for _ in range(1, spec.n_layers):
        out.append((_r8(act, off, rows, cols)[:, :spec.hidden] > 0).to(device))
        off += rp * cols
    return out


class MaskRecorder:
    """Install as graphphysics.models._engine.INSPECT; after a training forward, .masks holds the
    oracle-keyed masks {mlp prefix: [bool [rows, h]]} in the CALLER's row order (edge MLPs run in the
    target-sorted order: mapped back through csc_eid). device: where the masks are kept ("cpu", or the
    GPU for graphs whose masks would not fit the host comfortably — Cfg E: 8 GB of them)."""

    def __init__(self, device="cpu"):
        self.masks = None
        self.device = device

    def __call__(self, st):
        from graphphysics import _native as nat

        assert st["mdt"] == nat.MGN_F32, "mask pinning reads fp32 saves (bf16 rounds activations to 0)"
        assert not st.get("rew"), "the recomputed weight gradients save no edge-MLP layer inputs to read masks from"
        torch.cuda.synchronize()
        plan, topo = st["plan"], st["topo"]
        N, E = topo.num_nodes, topo.num_edges
        dev = self.device
        eid = topo.csc_eid[:E].long().to(dev)

        def to_caller(ms):
            out = []
            for m in ms:
                o = torch.empty_like(m)
                o[eid] = m
                out.append(o)
            return out

        masks = {}
        ks = 4
        if not st["only_processor"]:
            ne, ee, dec = plan.specs[:3]
            masks["nodes_encoder"] = _mlp_masks(ne, st["sv_ne"][1][0], N, False, ks, dev)
            masks["edges_encoder"] = to_caller(_mlp_masks(ee, st["sv_ee"][1][0], E, False, ks, dev))
            masks["decode_module"] = _mlp_masks(dec, st["sv_dec"][1][0], N, False, ks, dev)
            bspecs = plan.specs[3:]
        else:
            bspecs = plan.specs
        for b, sv in enumerate(st["svs"]):
            ke, kn, _ = sv[1]
            masks[f"processor_list.{b}.edge_block"] = to_caller(_mlp_masks(bspecs[2 * b], ke[0], E, True, ks, dev))
            masks[f"processor_list.{b}.node_block"] = _mlp_masks(bspecs[2 * b + 1], kn[0], N, True, ks, dev)
        self.masks = masks


class FlipStats(dict):
    """A `record=` sink for the oracle's mlp that keeps flip statistics instead of the pre-activations
    (graphs whose fp64 pre-activations would not fit: Cfg E, 1.4 GB per layer): per MLP layer, the count
    of units whose pinned branch differs from the fp64 sign and their largest |z64| / mean |z64|. The
    mlp appends its hidden layers' pre-activations in order (again when a checkpointed block is
    recomputed: the layer index is the append count modulo the hidden layers)."""

    def __init__(self, masks, hidden_layers=3):
        super().__init__()
        self._masks, self._nh, self._sinks = masks, hidden_layers, {}

    def setdefault(self, prefix, default=None):
        sink = self._sinks.get(prefix)
        if sink is None:
            stats = self

            class _Sink:
                count = 0

                def append(self, z):
                    i = self.count % stats._nh
                    self.count += 1
                    m = stats._masks[prefix][i]
                    d = m != (z > 0)
                    n = int(d.sum())
                    if n:
                        key = f"{prefix}.{2 * i}"
                        r = float(z[d].abs().max() / z.abs().mean())
                        old = dict.get(stats, key, {"flipped": 0, "max_rel_z": 0.0})
                        dict.__setitem__(stats, key, {"flipped": max(old["flipped"], n),
                                                      "max_rel_z": max(old["max_rel_z"], r)})

            sink = self._sinks[prefix] = _Sink()
        return sink


def flips(masks, record):
    """Units whose libmgn branch differs from the natural fp64 ReLU: per MLP layer, the count and
    the largest |z64| / mean |z64| of the layer among them (a near-tie is ≪ 1)."""
    out = {}
    for pre, zs in record.items():
        for i, z in enumerate(zs):
            m = masks[pre][i]
            d = m != (z > 0)
            n = int(d.sum())
            if n:
                out[f"{pre}.{2 * i}"] = {"flipped": n, "max_rel_z": float(z[d].abs().max() / z.abs().mean())}
    return out
