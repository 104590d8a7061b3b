"""fp32 gradient parity of the full 15-block model with the ReLU branches pinned.

Deep stacks hold pre-activations within fp32 rounding of 0: the reference's own fp32 path and libmgn
each put such a unit on one side of its ReLU, and whichever side moves every upstream gradient by up
to ~1e-3 (test_gpu_parity.py bounds that with the reference's summation-order spread). Here the tie
is taken out instead of bounded: the oracle (the reference's ops, oracle/mgn_oracle.py restating
layers.py:18-113,630-746 and processors.py:111-137) is evaluated in fp64 on the branch libmgn took
(tests/_masks.py reads it from libmgn's fp32 forward saves), and then
  * the output must be within rel-L2 1e-5 and EVERY parameter gradient within rel-L2 1e-3 (§8(c)) of
    that evaluation — rounding is all that is left, measured ~1e-6;
  * every unit where libmgn's branch differs from the fp64 sign must be a near-tie (|z64| ≤ 1e-4 of its
    layer's mean |z|): a kernel error would flip units with large |z| or move gradients on the pinned
    branch, a tie does neither. The flips are logged (MGN_TEST_RECORD_DIR/mask_flips.json).
Inputs: the CylinderFlow mesh at seed 7 (test_epd_cylinder_vs_oracle's input, the one round 3's fp32
chained kernels first failed the unpinned bound on), and Cfg B at its real batch (8 jittered copies:
N = 15,384, E = 88,560; batching as simulator.py:283-288 / torch_geometric Batch), also vs the CPU
fp32 oracle forward and, in bf16, vs PyTorch's own bf16 autocast of the reference algorithm.
"""
import json
import os

import pytest
import torch

from _masks import MaskRecorder, flips
from oracle import mgn_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _built():
    import __graft_entry__ as ge

    ge.build()
    assert torch.cuda.is_available(), "GPU tests need a HIP device"


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _graph(batch):
    from graphphysics.utils import meshes

    if batch == 1:
        m = meshes.load_cylinder_mesh()
        n = m["pos"].shape[0]
        return n, torch.from_numpy(meshes.triangles_to_edge_index(m["triangles"], n))
    b = meshes.cylinder_batch(batch, t=0, jitter=0.01, seed=1234)
    return b["x"].shape[0], torch.from_numpy(b["edge_index"])


def _inputs(batch):
    n, ei = _graph(batch)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(n, 11, generator=g)
    ea = torch.randn(ei.shape[1], 3, generator=g)
    gy = torch.randn(n, 2, generator=g)
    return n, ei, x, ea, gy


def _record(name, obj):
    d = os.environ.get("MGN_TEST_RECORD_DIR")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    f = os.path.join(d, "mask_flips.json")
    allr = json.load(open(f)) if os.path.exists(f) else {}
    allr[name] = obj
    json.dump(allr, open(f, "w"), indent=1)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mp,h,batch", [(5, 32, 1), (15, 128, 1), (15, 128, 8)])
def test_epd_fp32_mask_pinned_vs_fp64(mp, h, batch):
    from graphphysics.models import _engine
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.utils.data import Data

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    n, ei, x, ea, gy = _inputs(batch)
    torch.manual_seed(0)
    m = EncodeProcessDecode(mp, 11, 3, 2, h, compute_dtype=torch.float32).to(DEV)
    rec = MaskRecorder()
    _engine.INSPECT = rec
    try:
        y = m(Data(x=x.to(DEV), edge_index=ei.to(DEV), edge_attr=ea.to(DEV)))
    finally:
        _engine.INSPECT = None
    (y * gy.to(DEV)).sum().backward()
    assert rec.masks is not None and len(rec.masks) == 3 + 2 * mp

    # fp64 on libmgn's branch
    p64 = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.named_parameters()}
    zrec = {}
    y64 = O.encode_process_decode(x.double(), ei, ea.double(), p64, mp, masks=rec.masks, record=zrec)
    (y64 * gy.double()).sum().backward()
    fl = flips(rec.masks, zrec)
    errs = {k: relerr(p.grad, p64[k].grad) for k, p in m.named_parameters()}
    worst = max(errs, key=errs.get)
    _record(f"mp{mp}_h{h}_b{batch}", {"nodes": n, "edges": int(ei.shape[1]), "output_rel_l2": relerr(y, y64),
                                      "grad_rel_l2_max": errs[worst], "grad_rel_l2_worst_param": worst,
                                      "flips": fl})
    assert relerr(y, y64) <= 1e-5, relerr(y, y64)
    for k, e in errs.items():
        assert e <= 1e-3, f"{k}: libmgn fp32 {e:.2e} from the mask-pinned fp64 evaluation (SURVEY 8(c): 1e-3)"
    for k, v in fl.items():
        assert v["max_rel_z"] <= 1e-4, f"{k}: libmgn's branch differs from fp64 away from a tie: {v}"
    if batch > 1:
        # Cfg B at model level vs the reference's CPU fp32 path (the oracle's ops as ATen runs them)
        with torch.no_grad():
            p32 = {k: v.detach().cpu() for k, v in m.named_parameters()}
            yr = O.encode_process_decode(x, ei, ea, p32, mp)
        assert relerr(y, yr) <= 1e-4, relerr(y, yr)


@pytest.mark.timeout(600)
def test_epd_bf16_cfgB_batch8_vs_autocast():
    """Cfg B (BASELINE configs[1]: bf16, batch 8) at model level: libmgn bf16 no further from the fp64
    evaluation than 2x PyTorch's own bf16 autocast of the reference algorithm on the same inputs
    (output; every parameter gradient: max(1e-2, 2x autocast's))."""
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.utils.data import Data

    torch.set_num_threads(min(16, os.cpu_count() or 1))
    mp, h = 15, 128
    n, ei, x, ea, gy = _inputs(8)
    torch.manual_seed(0)
    m = EncodeProcessDecode(mp, 11, 3, 2, h, compute_dtype=torch.bfloat16).to(DEV)
    y = m(Data(x=x.to(DEV), edge_index=ei.to(DEV), edge_attr=ea.to(DEV)))
    (y * gy.to(DEV)).sum().backward()
    p64 = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.named_parameters()}
    y64 = O.encode_process_decode(x.double(), ei, ea.double(), p64, mp)
    (y64 * gy.double()).sum().backward()
    pac = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.named_parameters()}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        yac = O.encode_process_decode(x, ei, ea, pac, mp)
    (yac.float() * gy).sum().backward()
    e_out, e_ac = relerr(y, y64), relerr(yac, y64)
    ratios = {}
    for k, p in m.named_parameters():
        ratios[k] = relerr(p.grad, p64[k].grad) / max(relerr(pac[k].grad, p64[k].grad), 1e-30)
    _record("bf16_cfgB_b8", {"output_rel_l2": e_out, "autocast_output_rel_l2": e_ac,
                             "grad_ratio_median": float(torch.tensor(list(ratios.values())).median()),
                             "grad_ratio_max": max(ratios.values())})
    assert e_out <= 2 * e_ac, (e_out, e_ac)
    for k, p in m.named_parameters():
        assert relerr(p.grad, p64[k].grad) <= max(1e-2, 2 * relerr(pac[k].grad, p64[k].grad)), k
