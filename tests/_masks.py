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


def _mlp_masks(spec, act, rows, gathered, kstep):
    """[bool [rows, hidden] per hidden layer] of one MLP from its saved act buffer."""
    rp = _rows_pad(rows)
    cols = _rup(spec.width, kstep)
    off = 0 if gathered else rp * _rup(spec.shapes[0][1], kstep)
    out = []
    for _ in range(1, spec.n_layers):
        out.append((_r8(act, off, rows, cols)[:, :spec.hidden] > 0).cpu())
        off += rp * cols
    return out


class MaskRecorder:
    """Install as graphphysics.models._engine.INSPECT; after a training forward, .masks holds the
    oracle-keyed masks {mlp prefix: [bool [rows, h]]} in the CALLER's row order (edge MLPs run in the
    target-sorted order: mapped back through csc_eid)."""

    def __init__(self):
        self.masks = None

    def __call__(self, st):
        from graphphysics import _native as nat

        assert st["mdt"] == nat.MGN_F32, "mask pinning reads fp32 saves (bf16 rounds activations to 0)"
        torch.cuda.synchronize()
        plan, topo = st["plan"], st["topo"]
        N, E = topo.num_nodes, topo.num_edges
        eid = topo.csc_eid[:E].long().cpu()

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
            masks["nodes_encoder"] = _mlp_masks(ne, st["sv_ne"][1][0], N, False, ks)
            masks["edges_encoder"] = to_caller(_mlp_masks(ee, st["sv_ee"][1][0], E, False, ks))
            masks["decode_module"] = _mlp_masks(dec, st["sv_dec"][1][0], N, False, ks)
            bspecs = plan.specs[3:]
        else:
            bspecs = plan.specs
        for b, sv in enumerate(st["svs"]):
            ke, kn, _ = sv[1]
            masks[f"processor_list.{b}.edge_block"] = to_caller(_mlp_masks(bspecs[2 * b], ke[0], E, True, ks))
            masks[f"processor_list.{b}.node_block"] = _mlp_masks(bspecs[2 * b + 1], kn[0], N, True, ks)
        self.masks = masks


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
