"""GPU parity of the MGN model on the two single-GPU BASELINE configs beyond CylinderFlow
(SURVEY.md §8 Cfg C and Cfg E), against the oracle (the reference's ops on the CPU):

  Cfg C  DeformingPlate MGN (reference training_config/plate.json:9-36 with type = epd): a plate-shaped
         tet mesh + obstacle (meshes.plate_sample, ~1.35k nodes) through the reference's world-pos
         preprocessing on the device (add_obstacles_next_pos, FaceToEdge, add_world_edges r = 0.03,
         Cartesian + Distance, world-pos features: preprocessing.py:49-174) -> node_in 6 + 9 = 15,
         edge_in 8, out 3, MP = 15, h = 128; the whole Simulator training forward + backward.
  Cfg E  3D aneurysm (reference coarse-aneurysm.json:9-24, torch_graph.py:16-110): the in-tree mock
         mesh, k-hop 2 built on the device (N = 22,535, E = 1,395,256, max in-degree 103), node_in
         14 + 9 = 23, edge_in 4, out 3, MP = 15, h = 128.

Tolerances (as tests/test_gpu_parity.py): fp32 forward rel-L2 <= 1e-4 for the full
15-block model and elementwise <= 1e-5(1 + |ref|) for the preamble; fp32 gradients no further from
the fp64 evaluation than max(2 x the reference fp32 path's own error, 2e-3 ReLU-tie floor); bf16 no
further from fp64 than 2 x PyTorch's CPU bf16 autocast of the reference (full model) or rel-L2 <=
1e-2 forward / 1.5e-1 gradients (single block); the fp32 segmented sum at in-degree 103 bit-exact
against ATen's scatter_add_ (same visiting order).
"""
import os

import numpy as np
import pytest
import torch

from oracle import mgn_oracle as O
from _orders import assert_vs_truth_orders, order_spread

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _built():
    import __graft_entry__ as ge

    ge.build()
    assert torch.cuda.is_available(), "GPU tests need a HIP device"


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def assert_close_elem(got, ref, tol=1e-5):
    got, ref = got.detach().double().cpu(), ref.detach().double().cpu()
    bad = (got - ref).abs() > tol * (1 + ref.abs())
    assert not bad.any(), f"max err {(got - ref).abs().max().item()}"


# ----------------------------------------------------------------------------- Cfg C: DeformingPlate
@pytest.fixture(scope="module")
def plate():
    from graphphysics.utils import meshes

    g, lay = meshes.plate_graph(DEV, seed=0)
    return g, lay


def _oracle_sim(model, lay):
    return O.OracleSimulator(model, lay["node_in"], lay["edge_in"], lay["out"], feature_slice=lay["fs"],
                             output_slice=lay["os"], node_type_index=lay["nti"])


def _sim(lay, dtype, mp=15, h=128):
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator

    torch.manual_seed(0)
    m = EncodeProcessDecode(mp, lay["node_in"], lay["edge_in"], lay["out"], h, compute_dtype=dtype)
    return Simulator(lay["node_in"], lay["edge_in"], lay["out"], lay["fs"][0], lay["fs"][1], lay["os"][0],
                     lay["os"][1], lay["nti"], m, DEV)


def test_plate_graph_shapes(plate):
    """Cfg C input contract: node features 6 + one-hot 9, edge_attr 8 (Cartesian 3 + Distance 1 +
    relative world pos 3 + norm 1), world edges present, edge_index coalesced and symmetric."""
    from graphphysics.utils import meshes

    g, lay = plate
    s = meshes.plate_sample(seed=0)
    n = s["x"].shape[0]
    assert g.x.shape == (n, 7) and g.y.shape == (n, 3) and g.edge_attr.shape == (g.edge_index.shape[1], 8)
    ei = g.edge_index.cpu()
    mesh_only = 0
    from oracle import graph_oracle as GO

    mesh_only = GO.face_to_edge(torch.from_numpy(s["cells"]).t().contiguous(), n).shape[1]
    assert ei.shape[1] > mesh_only  # world edges between the obstacle and the plate
    key = ei[0] * n + ei[1]
    assert torch.equal(key, key.sort().values) and torch.unique(key).numel() == key.numel()
    rev = torch.sort(ei[1] * n + ei[0]).values
    assert torch.equal(rev, key)


@pytest.mark.parametrize("mp,h", [(15, 128), (10, 64)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_plate_simulator_train_step_vs_oracle(plate, dtype, mp, h):
    """Cfg C: Simulator training forward (preamble + EPD) and backward of the masked L2 loss through
    libmgn vs the oracle on the same preprocessed plate graph — at the headline model size (MP=15,
    h=128) and at plate.json's own (message_passing_num 10, hidden_size 64: training_config/plate.json)."""
    from graphphysics.utils.loss import masked_mse
    from graphphysics.utils.nodetype import NodeType

    g, lay = plate
    sim = _sim(lay, dtype, mp, h)
    net, tdn, _ = sim(g)
    masks = [NodeType.NORMAL, NodeType.OUTFLOW]
    loss = masked_mse(tdn, net, g.x[:, lay["nti"]], masks)
    loss.backward()
    torch.cuda.synchronize()

    torch.manual_seed(0)
    ref = O.OracleEPD(mp, lay["node_in"], lay["edge_in"], lay["out"], h)
    osim = _oracle_sim(ref, lay)
    x, y, ei, ea = g.x.cpu(), g.y.cpu(), g.edge_index.cpu(), g.edge_attr.cpu()
    # the preamble (target delta, one-hot, three normalizers) against the reference's ops
    pre = x[:, 0:3]
    tdn_r = osim.out_norm(y - pre, True)
    onehot = torch.nn.functional.one_hot(x[:, lay["nti"]].long(), 9)
    nfn_r = osim.node_norm(torch.cat([x[:, 0:6], onehot], 1), True)
    ean_r = osim.edge_norm(ea, True)
    assert_close_elem(tdn, tdn_r)
    rp = dict(ref.named_parameters())
    yr = O.encode_process_decode(nfn_r, ei, ean_r, rp, mp)
    nt = x[:, lay["nti"]]
    lr = O.l2_loss(tdn_r, yr, nt)
    lr.backward()
    p64 = {k: v.detach().double().requires_grad_(True) for k, v in rp.items()}
    y64 = O.encode_process_decode(nfn_r.double(), ei, ean_r.double(), p64, mp)
    O.l2_loss(tdn_r.double(), y64, nt).backward()
    if dtype == torch.float32:
        assert relerr(net, yr) < 1e-4
        assert relerr(net, y64) <= max(1e-6, 2 * relerr(yr, y64))
        assert abs(loss.item() - lr.item()) <= 1e-4 * lr.item()
        sp = order_spread(lambda q, i: O.l2_loss(tdn_r, O.encode_process_decode(i["x"], ei, i["ea"], q, mp), nt), rp,
                          {k: v.grad for k, v in p64.items()}, n_orders=24,
                          inputs={"x": (nfn_r, "nodes_encoder.0.weight"), "ea": (ean_r, "edges_encoder.0.weight")})
        for k, p in sim.model.named_parameters():
            assert_vs_truth_orders(p.grad, rp[k].grad, p64[k].grad, sp[k], what=k)
        return
    pac = {k: v.detach().clone().requires_grad_(True) for k, v in rp.items()}
    with torch.autocast("cpu", dtype=torch.bfloat16):
        yac = O.encode_process_decode(nfn_r, ei, ean_r, pac, mp)
    O.l2_loss(tdn_r, yac.float(), nt).backward()
    assert relerr(net, y64) <= 2 * relerr(yac, y64)
    for k, p in sim.model.named_parameters():
        assert relerr(p.grad, p64[k].grad) <= max(1e-2, 2 * relerr(pac[k].grad, p64[k].grad)), k


# ----------------------------------------------------------------------------- Cfg E: aneurysm k-hop 2
def _aneurysm(khop):
    from graphphysics.utils import graph_build as G

    z = np.load(os.path.join(ROOT, "tests", "golden", "aneurysm_mesh.npz"))
    pos = torch.from_numpy(z["pos"]).to(DEV)
    tet = torch.from_numpy(z["tetra"].astype(np.int64)).t().contiguous().to(DEV)
    n = pos.shape[0]
    ei = G.face_to_edge(tet, n)
    if khop > 1:
        ei = G.k_hop_edge_index(ei, khop, n)
    ea = G.edge_features(pos, ei)
    rng = np.random.default_rng(1234)
    feats = rng.standard_normal((n, 14)).astype(np.float32)
    nt = rng.choice([0, 4, 5, 6], size=n, p=[0.9, 0.01, 0.01, 0.08]).astype(np.float32)
    x = torch.from_numpy(np.concatenate([feats, nt[:, None]], 1))
    y = torch.from_numpy((feats[:, 0:3] + 0.01 * rng.standard_normal((n, 3))).astype(np.float32))
    return n, ei, ea, x, y


@pytest.fixture(scope="module")
def aneurysm():
    return _aneurysm(2)


def test_aneurysm_graph_is_cfg_e(aneurysm):
    n, ei, ea, x, y = aneurysm
    assert (n, ei.shape[1]) == (22535, 1395256)
    deg = torch.bincount(ei[1].cpu(), minlength=n)
    assert int(deg.max()) == 103 and ea.shape == (1395256, 4)


def test_aneurysm_segment_sum_degree_103_bitexact(aneurysm):
    """fp32 segmented sum over the target-sorted in-edges at in-degree up to 103 (mgn_segment_sum on
    the block topology) equals ATen's scatter_add_ over edge_index[1] bit for bit: the coalesced
    (row, col) order visits each target's in-edges in increasing source order, as the CSC order does."""
    from graphphysics import _native as nat
    from graphphysics.models import _engine

    n, ei, ea, x, y = aneurysm
    E = ei.shape[1]
    topo = _engine.get_topology(ei, n)
    g = torch.Generator().manual_seed(3)
    m = torch.randn(E, 128, generator=g)
    ref = torch.zeros(n, 128).scatter_add_(0, ei[1].cpu()[:, None].expand(-1, 128), m)
    md = m.to(DEV)
    msorted = _engine._permute(md, topo.csc_eid, E, 128, nat.MGN_F32, torch.float32, False,
                               nat.stream_ptr(DEV))
    out = torch.empty(n, 128, device=DEV)
    nat.check(nat.lib().mgn_segment_sum(nat.ptr(msorted), nat.ptr(topo.col_ptr), n, 128, nat.MGN_F32,
                                        nat.ptr(out), nat.stream_ptr(DEV)))
    assert torch.equal(out.cpu(), ref)


def test_aneurysm_block_bf16_chained_degree_103_vs_fp64(aneurysm):
    """One bf16 h=128 GraphNetBlock on the Cfg E graph: the chained node kernel aggregates 103 in-edges
    per node in batches (MGN_NODE_AG per round trip); forward and gradients vs the fp64 oracle block
    on the same bf16-representable inputs (single-block bf16 bounds)."""
    from graphphysics.models.layers import GraphNetBlock

    n, ei, ea, x, y = aneurysm
    E = ei.shape[1]
    g = torch.Generator().manual_seed(5)
    xb = torch.randn(n, 128, generator=g).bfloat16().float()
    eb = torch.randn(E, 128, generator=g).bfloat16().float()
    gx = torch.randn(n, 128, generator=g)
    ge = torch.randn(E, 128, generator=g)
    torch.manual_seed(0)
    blk = GraphNetBlock(128)
    blk.compute_dtype = torch.bfloat16
    rp = {k: v.detach().double().requires_grad_(True) for k, v in blk.named_parameters()}
    blk = blk.to(DEV)
    xd = xb.to(DEV).requires_grad_(True)
    ed = eb.to(DEV).requires_grad_(True)
    x1, e1 = blk(xd, ei, ed)
    ((x1.float() * gx.to(DEV)).sum() + (e1.float() * ge.to(DEV)).sum()).backward()
    torch.cuda.synchronize()
    x64 = xb.double().requires_grad_(True)
    e64 = eb.double().requires_grad_(True)
    xr, er = O.graph_net_block(x64, ei.cpu(), e64, rp, "")
    ((xr * gx.double()).sum() + (er * ge.double()).sum()).backward()
    assert relerr(x1, xr) <= 1e-2 and relerr(e1, er) <= 1e-2
    assert relerr(xd.grad, x64.grad) <= 1.5e-1 and relerr(ed.grad, e64.grad) <= 1.5e-1
    for k, p in blk.named_parameters():
        assert relerr(p.grad, rp[k].grad) <= 1.5e-1, k


def test_aneurysm_simulator_fp32_forward_full_size(aneurysm):
    """Cfg E at full size, fp32: Simulator training-mode forward (preamble + 15-block EPD) through
    libmgn vs the oracle — full-model rel-L2 <= 1e-4 and no further from fp64... (fp64 at 4.3 TFLOP is
    skipped at this size; the fp32 oracle is the reference's own arithmetic)."""
    from graphphysics.utils.data import Data

    n, ei, ea, x, y = aneurysm
    lay = dict(node_in=23, edge_in=4, out=3, fs=(0, 14), os=(0, 3), nti=14)
    sim = _sim(lay, torch.float32)
    with torch.no_grad():
        net, tdn, _ = sim(Data(x=x.to(DEV), y=y.to(DEV), edge_index=ei, edge_attr=ea))
    torch.cuda.synchronize()
    torch.manual_seed(0)
    ref = O.OracleEPD(15, 23, 4, 3, 128)
    osim = _oracle_sim(ref, lay)
    with torch.no_grad():
        nr, tr, _ = osim.forward(x, y, ei.cpu(), ea.cpu(), True)
    assert_close_elem(tdn, tr)
    assert relerr(net, nr) < 1e-4


# ----------------------------------------------------------------------------- Cfg E at full size
# The fp32 / fp64 / bf16-autocast evaluations of the reference algorithm at this size (4.3 TFLOP per
# forward at MP=15) take minutes on the host, so these tests evaluate the ORACLE's functional core
# (oracle/mgn_oracle.py: the reference's ATen op sequence — index, cat, addmm, scatter_add_, ...)
# through PyTorch's own ROCm kernels on the GPU, not through libmgn, with per-block recomputation
# (torch.utils.checkpoint) to bound memory. PyTorch's fp32 GPU path plays the part of "the
# reference's fp32 path" (a different summation order — scatter_add_ by atomics — but the same
# fp32 arithmetic class); its error against fp64 sets the bound as on the CPU.
def _epd_ckpt(x, ei, e, p, mp):
    from torch.utils.checkpoint import checkpoint

    x = O.mlp(x, p, "nodes_encoder")
    e = O.mlp(e, p, "edges_encoder")
    for b in range(mp):
        x, e = checkpoint(O.graph_net_block, x, ei, e, p, f"processor_list.{b}.", use_reentrant=False)
    return O.mlp(x, p, "decode_module", norm=False)


def _aten_eval(ref, x, ei, ea, gy, mp, dtype, autocast=False):
    """Output and gradients (parameters, x, edge_attr) of sum(EPD(x) * gy) by the oracle's ops on the GPU."""
    p = {k: v.detach().to(DEV, dtype).requires_grad_(True) for k, v in ref.named_parameters()}
    xd = x.to(DEV, dtype).requires_grad_(True)
    ed = ea.to(DEV, dtype).requires_grad_(True)
    if autocast:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = _epd_ckpt(xd, ei, ed, p, mp)
    else:
        y = _epd_ckpt(xd, ei, ed, p, mp)
    keys = list(p)
    grads = torch.autograd.grad((y.to(gy.dtype) * gy).sum(), [xd, ed] + [p[k] for k in keys])
    torch.cuda.synchronize()
    out = {"y": y.detach().double().cpu(), "x": grads[0].double().cpu(), "e": grads[1].double().cpu()}
    out.update({k: g.double().cpu() for k, g in zip(keys, grads[2:])})
    del p, xd, ed, y, grads
    torch.cuda.empty_cache()
    return out


def _libmgn_eval(x, ei, ea, gy, mp, h, dtype, node_in, edge_in, out, masks=None):
    """masks (a tests/_masks.MaskRecorder): record the ReLU branch of every hidden unit libmgn took."""
    from graphphysics.models import _engine
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.utils.data import Data

    torch.manual_seed(0)
    m = EncodeProcessDecode(mp, node_in, edge_in, out, h, compute_dtype=dtype).to(DEV)
    xd = x.to(DEV).detach().clone().requires_grad_(True)  # fresh leaves: never the fixture's tensors
    ed = ea.to(DEV).detach().clone().requires_grad_(True)
    _engine.INSPECT = masks
    try:
        y = m(Data(x=xd, edge_index=ei, edge_attr=ed))
    finally:
        _engine.INSPECT = None
    (y * gy.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    res = {"y": y.detach().double().cpu(), "x": xd.grad.double().cpu(), "e": ed.grad.double().cpu()}
    res.update({k: v.grad.double().cpu() for k, v in m.named_parameters()})
    del m, xd, ed, y
    torch.cuda.empty_cache()
    return res


def _rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-300))


def _pinned_eval(ref, x, ei, ea, gy, mp, masks, stats):
    """_aten_eval in fp64 on libmgn's ReLU branch (tests/_masks.py; checkpointed blocks)."""
    from torch.utils.checkpoint import checkpoint

    p = {k: v.detach().to(DEV, torch.float64).requires_grad_(True) for k, v in ref.named_parameters()}
    xd = x.to(DEV, torch.float64).requires_grad_(True)
    ed = ea.to(DEV, torch.float64).requires_grad_(True)
    kw = dict(masks=masks, record=stats)
    xe = O.mlp(xd, p, "nodes_encoder", **kw)
    e = O.mlp(ed, p, "edges_encoder", **kw)
    for b in range(mp):
        xe, e = checkpoint(O.graph_net_block, xe, ei, e, p, f"processor_list.{b}.", masks, stats, use_reentrant=False)
    y = O.mlp(xe, p, "decode_module", norm=False, **kw)
    keys = list(p)
    grads = torch.autograd.grad((y * gy.to(DEV, torch.float64)).sum(), [xd, ed] + [p[k] for k in keys])
    torch.cuda.synchronize()
    out = {"y": y.detach().cpu(), "x": grads[0].cpu(), "e": grads[1].cpu()}
    out.update({k: g.cpu() for k, g in zip(keys, grads[2:])})
    del p, xd, ed, y, grads
    torch.cuda.empty_cache()
    return out


@pytest.mark.parametrize("khop,mp,h", [(2, 15, 128), (1, 10, 64)])
def test_aneurysm_full_size_fp32_and_bf16_gradients(khop, mp, h):
    """Cfg E at full size: the 3D aneurysm graph with k-hop 2 (E = 1,395,256, in-degree up to 103) and
    the headline model (MP=15, h=128), and coarse-aneurysm.json's own sizes (k-hop 1, MP=10, h=64:
    training_config/coarse-aneurysm.json); inputs node_in 23, edge_in 4, out 3.
      fp32: output rel-L2 <= 1e-4 vs the fp32 evaluation; output (1e-5), every parameter gradient and
            the input gradients (x, edge_attr) within SURVEY §8c's 1e-3 of the fp64 evaluation on
            libmgn's ReLU branch (mask-pinned), every flipped unit a near-tie; AND, unpinned (VERDICT
            r05 item 2: so libmgn's fp32 cannot drift from the reference's own fp32 distance to fp64),
            every gradient within max(1.5e-3, 2 x the worst error the reference algorithm's fp32 shows
            vs the unpinned fp64 evaluation over PyTorch's own order and 4 permuted summation orders
            (tests/_orders.py order_spread)). The 1.5e-3 floor: near-ties flipped by any fp32 order move
            upstream gradients by up to ~1e-3 (measured round 5: libmgn 1.06e-3 on block 12's edge W0,
            PyTorch's fp32 2.5e-4 / 3.8e-4 in two runs), 4 orders need not sample the same tie, and
            4 x 1.4M-edge fp32 orders is what the test budget holds (the Cfg B checks run 24).
      bf16: output and every gradient no further from fp64 than 2 x the bf16 autocast evaluation's
            error (floor 1e-2), and the SAME on the rows of the highest in-degree nodes alone (nodes with
            in-degree >= the 99th percentile): an indexing error confined to long segments would stand out
            there while averaging away in the whole-tensor norm."""
    from _masks import FlipStats, MaskRecorder

    n, ei, ea, x, y = _aneurysm(khop)
    g = torch.Generator().manual_seed(21)
    xin = torch.randn(n, 23, generator=g)
    gy = torch.randn(n, 3, generator=g)
    torch.manual_seed(0)
    ref = O.OracleEPD(mp, 23, 4, 3, h)
    r64 = _aten_eval(ref, xin, ei, ea.cpu(), gy.to(DEV, torch.float64), mp, torch.float64)
    r32 = _aten_eval(ref, xin, ei, ea.cpu(), gy.to(DEV), mp, torch.float32)
    rec = MaskRecorder(device=DEV)
    g32 = _libmgn_eval(xin, ei, ea, gy, mp, h, torch.float32, 23, 4, 3, masks=rec)
    assert _rel(g32["y"], r32["y"]) <= 1e-4
    # fp32 gradients vs fp64 ON libmgn's ReLU branch (as tests/test_mask_pinned_gpu.py for Cfg B): 15
    # blocks of 1.4M edges hold pre-activations within fp32 rounding of 0, which any fp32 summation order
    # — PyTorch's atomics included — puts on either side of a ReLU, moving every upstream gradient by up
    # to ~1e-3 (round 5: a reordered fp32 node-MLP GEMM moved block 12's edge W0 gradient to 1.07e-3 of
    # the unpinned fp64 evaluation while PyTorch's own fp32 run sat at 2.5e-4 / 3.8e-4 in two runs).
    # Pinned, what is left is rounding: every gradient within SURVEY §8(c)'s 1e-3, and every unit whose
    # branch differs from the fp64 sign a near-tie (|z64| <= 1e-4 of its layer's mean |z|).
    stats = FlipStats(rec.masks)
    p64 = _pinned_eval(ref, xin, ei, ea, gy, mp, rec.masks, stats)
    del rec
    assert _rel(g32["y"], p64["y"]) <= 1e-5, _rel(g32["y"], p64["y"])
    # the reference algorithm's fp32 spread vs the unpinned fp64 evaluation, in 4 more summation orders
    gy32 = gy.to(DEV)
    rp = {k: v.detach().to(DEV, torch.float32) for k, v in ref.named_parameters()}
    sp = order_spread(lambda q, i: (_epd_ckpt(i["x"], ei, i["ea"], q, mp) * gy32).sum(), rp,
                      {k: r64[k] for k in rp}, n_orders=4, seed=5,
                      inputs={"x": (xin.to(DEV), "nodes_encoder.0.weight"),
                              "ea": (ea.to(DEV).float(), "edges_encoder.0.weight")})
    del rp
    torch.cuda.empty_cache()
    worst, worst_u = [], []
    for k in p64:
        e_got, e_unpinned, e_ref = _rel(g32[k], p64[k]), _rel(g32[k], r64[k]), _rel(r32[k], r64[k])
        worst.append((e_got, k, e_unpinned, e_ref))
        assert e_got <= 1e-3, (k, e_got, e_unpinned, e_ref)
        bound = max(1.5e-3, 2 * max(e_ref, sp.get(k, 0.0)))
        worst_u.append((e_unpinned / bound, k, e_unpinned, e_ref, sp.get(k)))
        assert e_unpinned <= bound, ("unpinned", k, e_unpinned, e_ref, sp.get(k))
    print("\nfp32 worst pinned (libmgn vs pinned fp64, key, vs unpinned fp64, aten-fp32 vs fp64):", sorted(worst)[-3:])
    print("fp32 worst unpinned (ratio to bound, key, libmgn, aten-fp32, worst permuted order):", sorted(worst_u)[-3:])
    print("fp32 branch flips:", dict(stats))
    for k, v in stats.items():
        assert v["max_rel_z"] <= 1e-4, f"{k}: libmgn's branch differs from fp64 away from a tie: {v}"
    del g32, r32, p64
    rac = _aten_eval(ref, xin, ei, ea.cpu(), gy.to(DEV), mp, torch.float32, autocast=True)
    gbf = _libmgn_eval(xin, ei, ea, gy, mp, h, torch.bfloat16, 23, 4, 3)
    deg = torch.bincount(ei[1].cpu(), minlength=n)
    hi = deg >= torch.quantile(deg.double(), 0.99)
    worst = []
    for k in r64:
        e_got, e_ac = _rel(gbf[k], r64[k]), _rel(rac[k], r64[k])
        worst.append((e_got / max(1e-2, 2 * e_ac), k, e_got, e_ac))
        assert e_got <= max(1e-2, 2 * e_ac), (k, e_got, e_ac)
    for k in ("y", "x"):
        e_got, e_ac = _rel(gbf[k][hi], r64[k][hi]), _rel(rac[k][hi], r64[k][hi])
        assert e_got <= max(1e-2, 2 * e_ac), ("high in-degree rows", k, e_got, e_ac)
    print("bf16 worst (ratio, key, libmgn, autocast):", sorted(worst)[-3:])
