"""Host-side logic of the drop-in package, on CPU (no kernels): module structure / state_dict
compatibility with the reference, RNG-order parity of initialisation, flat parameter storage,
normaliser / loss / scheduler semantics against the oracle and golden vectors, mesh construction."""
import os

import numpy as np
import pytest
import torch

from oracle import mgn_oracle as O

G = os.path.join(os.path.dirname(__file__), "golden")


def _golden(name):
    z = np.load(os.path.join(G, name))
    return {k: z[k] for k in z.files}


def test_epd_state_dict_keys_and_init_match_reference():
    from graphphysics.models.processors import EncodeProcessDecode

    z = _golden("cylinder_golden.npz")
    for tag, mp, h in (("cfgA_init", 5, 32), ("cfgB_init", 15, 128)):
        torch.manual_seed(0)
        m = EncodeProcessDecode(mp, 11, 3, 2, h)
        sd = m.state_dict()
        pre = tag + "::model."
        ref_keys = sorted(k[len(pre):] for k in z if k.startswith(pre))
        assert sorted(sd) == ref_keys
        for k, v in sd.items():
            assert v.double().sum().item() == float(z[f"{tag}::model.{k}"]), k
    assert (m.K, m.d, m.temperature, m.hidden_size, m.only_processor) == (0, 2, None, 128, False)


def test_golden_weights_load_into_drop_in_modules():
    from graphphysics.models.layers import GraphNetBlock
    from graphphysics.models.processors import EncodeProcessDecode

    z = _golden("block_cycle_h16.npz")
    GraphNetBlock(16).load_state_dict({k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("w::")})
    z = _golden("epd_random_h16.npz")
    EncodeProcessDecode(3, 8, 4, 3, 16).load_state_dict(
        {k[3:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("w::")})


def test_flat_parameters_and_plan_order():
    from graphphysics.models import _engine
    from graphphysics.models.processors import EncodeProcessDecode

    m = EncodeProcessDecode(3, 11, 3, 2, 32)
    flat = m._flat_params
    o = 0
    for p in m.parameters():
        assert p.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()
        assert p.storage_offset() == o
        o += p.numel()
    assert o == flat.numel()
    m = m.double().float()  # _apply re-homes parameters into a fresh flat buffer
    assert all(p.untyped_storage().data_ptr() == m._flat_params.untyped_storage().data_ptr()
               for p in m.parameters())
    plan = m._get_plan()
    assert [s.in_dim for s in plan.specs[:3]] == [11, 3, 32]
    assert [s.out_dim for s in plan.specs[:3]] == [32, 32, 2]
    assert plan.specs[2].norm is None and plan.specs[3].norm is not None
    assert plan.offsets[1] == plan.specs[0].numel
    assert plan.numel == sum(p.numel() for p in m.parameters())
    g = torch.arange(plan.numel, dtype=torch.float32)
    views = plan.grad_views(g)
    assert [v.shape for v in views] == [p.shape for p in m.parameters()]
    with pytest.raises(ValueError):
        _engine.MlpSpec(torch.nn.Sequential(torch.nn.Linear(3, 4), torch.nn.Tanh(), torch.nn.Linear(4, 4)))


def test_gmm_heads_are_rejected_loudly():
    from graphphysics.models.processors import EncodeProcessDecode

    with pytest.raises(NotImplementedError):
        EncodeProcessDecode(2, 11, 3, 2, 16, num_mixture_components=2, temperature=1.0)


def test_normalizer_matches_reference_semantics():
    from graphphysics.models.layers import Normalizer

    g = torch.Generator().manual_seed(0)
    mine = Normalizer(5, max_accumulations=3, device="cpu")
    ref = O.OracleNormalizer(5, max_accumulations=3)
    for i in range(5):  # crosses max_accumulations: accumulation must stop
        d = torch.randn(17 + i, 5, generator=g) * 3 + 1
        a, b = mine(d, True), ref(d, True)
        assert torch.equal(a, b)
    assert torch.equal(mine.inverse(a), ref.inverse(a))
    assert mine._num_accumulations.item() == 3
    assert torch.equal(mine._acc_sum, ref.acc_sum)
    e = torch.randn(4, 5, generator=g)
    assert torch.equal(mine(e, False), ref(e, False))


class _ZeroModel(torch.nn.Module):
    K = 0

    def forward(self, graph):
        return torch.zeros(graph.x.shape[0], 2) + graph.x[:, :2].sum() * 0


def test_simulator_preamble_matches_reference():
    from graphphysics.models.simulator import Simulator
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    b = meshes.cylinder_batch(2)
    x, y = torch.from_numpy(b["x"]), torch.from_numpy(b["y"])
    ei, ea = torch.from_numpy(b["edge_index"]), torch.from_numpy(b["edge_attr"])
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, _ZeroModel(), "cpu")
    ref = O.OracleSimulator(lambda xn, e_, ean: torch.zeros(xn.shape[0], 2), 11, 3, 2)
    # host tensors never take the fused libmgn preamble (mgn_simulator_preamble needs HIP tensors)
    assert not sim._fused_preamble_ok(Data(x=x, y=y, edge_index=ei, edge_attr=ea), True)
    for _ in range(2):
        _, tdn, _ = sim(Data(x=x, y=y, edge_index=ei, edge_attr=ea))
        _, tdn_r, _ = ref.forward(x, y, ei, ea, True)
        assert torch.equal(tdn, tdn_r)
    assert torch.equal(sim._node_normalizer._acc_sum, ref.node_norm.acc_sum)
    assert torch.equal(sim._edge_normalizer._acc_sum_squared, ref.edge_norm.acc_sum_squared)
    sim.eval()
    _, _, out = sim(Data(x=x, y=y, edge_index=ei, edge_attr=ea))
    _, _, out_r = ref.forward(x, y, ei, ea, False)
    assert torch.equal(out, out_r)


def test_losses():
    from graphphysics.utils.loss import L2Loss, masked_mse
    from graphphysics.utils.nodetype import NodeType

    g = torch.Generator().manual_seed(0)
    t, o = torch.randn(100, 2, generator=g), torch.randn(100, 2, generator=g)
    nt = torch.randint(0, 7, (100,), generator=g).float()
    masks = [NodeType.NORMAL, NodeType.OUTFLOW]
    ref = O.l2_loss(t, o, nt)
    assert torch.equal(L2Loss()(t, o, nt, masks), ref)
    torch.testing.assert_close(masked_mse(t, o, nt, masks), ref, rtol=1e-6, atol=0)


def test_scheduler_matches_golden():
    from graphphysics.utils.scheduler import CosineWarmupScheduler

    z = _golden("cylinder_golden.npz")
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=1e-3)
    sch = CosineWarmupScheduler(opt, warmup=5, max_iters=100)
    lrs = []
    for _ in range(3):
        opt.step()
        sch.step()
        lrs.append(opt.param_groups[0]["lr"])
    np.testing.assert_array_equal(np.array(lrs), z["cfgA/lrs"])


def test_mesh_construction_pins():
    from graphphysics.utils import meshes

    m = meshes.load_cylinder_mesh()
    n = m["pos"].shape[0]
    ei = meshes.triangles_to_edge_index(m["triangles"], n)
    assert ei.shape == (2, 11070)
    # k-hop=2 count pinned by reference tests/graphphysics/dataset/test_xdmfdataset.py:228-230
    assert meshes.khop_edge_index(ei, n, 2).shape == (2, 32638)
    b = meshes.cylinder_batch(8)
    assert b["x"].shape == (15384, 3) and b["edge_index"].shape == (2, 88560)
    assert (np.diff(b["edge_index"][0]) >= 0).all()  # batching keeps (row, col) order


def test_product_path_refuses_cpu_tensors():
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.utils.data import Data

    m = EncodeProcessDecode(1, 5, 3, 2, 16)
    with pytest.raises(RuntimeError, match="HIP device"):
        m(Data(x=torch.zeros(4, 5), edge_index=torch.zeros((2, 1), dtype=torch.long),
               edge_attr=torch.zeros(1, 3)))


def test_pending_statistics_feed_one_forward_only():
    """exchanged (pending) statistics are consumed by exactly one accumulating forward;
    a second forward without a new exchange raises instead of silently re-adding them, and leaving
    data-parallel mode clears them."""
    from graphphysics.models.layers import Normalizer

    n = Normalizer(3, device="cpu")
    d = torch.randn(5, 3)
    n.set_pending(d.sum(0, keepdim=True), (d ** 2).sum(0, keepdim=True), torch.tensor(5.0))
    n(d)
    with pytest.raises(RuntimeError, match="already consumed"):
        n(d)
    n(d, accumulate=False)  # evaluation never consumes
    n.set_pending(d.sum(0, keepdim=True), (d ** 2).sum(0, keepdim=True), torch.tensor(5.0))
    n(d)
    n.clear_pending()
    n(d)  # local statistics again
    assert float(n._acc_count) == 15.0


def test_load_checkpoint_updates_normalizer_buffers_in_place(tmp_path):
    """load_checkpoint copies the normalizer statistics into the existing buffers, so a
    captured step / rollout graph recorded before the load reads the loaded values."""
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator

    def make():
        torch.manual_seed(0)
        return Simulator(11, 3, 2, 0, 2, 0, 2, 2, EncodeProcessDecode(2, 11, 3, 2, 8), torch.device("cpu"),
                         model_dir=str(tmp_path / "sim.pth"))

    a = make()
    for nrm in a.normalizers():
        nrm._acc_sum.uniform_()
        nrm._acc_count.fill_(7.0)
    a.save_checkpoint()
    b = make()
    before = [(nrm._acc_sum, nrm._acc_count) for nrm in b.normalizers()]
    b.load_checkpoint()
    for (s0, c0), na, nb in zip(before, a.normalizers(), b.normalizers()):
        assert nb._acc_sum is s0 and nb._acc_count is c0
        assert torch.equal(nb._acc_sum, na._acc_sum) and float(nb._acc_count) == 7.0


@pytest.mark.parametrize("h", [48, 96, 100, 128, 192, 256])
def test_padded_plan_layout_round_trips(h):
    """Hidden sizes the kernels are not instantiated for run zero-padded to the next kernel width
    (_engine.kernel_width): the padded parameter layout the kernels write gradients in must map
    back onto the true layout exactly (ModelPlan.unpad), and the packed shapes cover the model."""
    from graphphysics.models import _engine
    from graphphysics.models.processors import EncodeProcessDecode

    torch.manual_seed(0)
    m = EncodeProcessDecode(2, 11, 3, 2, h)
    plan = m._get_plan()
    W = _engine.kernel_width(h)
    assert plan.padded == (W != h)
    assert all(s.width == W for s in plan.specs)
    if not plan.padded:
        assert plan.numel_pad == plan.numel and plan.offsets_pad == plan.offsets
        return
    # a padded gradient buffer holding each true element at its padded position (and junk elsewhere)
    true = torch.arange(plan.numel, dtype=torch.float32)
    gp = torch.full((plan.numel_pad,), -1.0)
    gp[plan._unpad_cpu] = true
    assert torch.equal(plan.unpad(gp), true)
    assert torch.unique(plan._unpad_cpu).numel() == plan.numel and int(plan._unpad_cpu.max()) < plan.numel_pad
    blk = plan.specs[3]  # block 0's edge MLP: layer 0 = [e ‖ x_i ‖ x_j], three h-blocks each padded to W
    assert blk.shapes[0][:2] == (W, 3 * W) and blk.shapes[0][4:] == (h, W)
    dec = plan.specs[2]
    assert dec.shapes[-1][:2] == (2, W) and dec.out_width == 2
    # the decoder reads the padded hidden state: its layer 0 (and so its input gradient, which the
    # processor's last block reads W wide) is W wide
    assert dec.shapes[0][:2] == (W, W) and dec.shapes[0][4:] == (h, W)
    enc = plan.specs[0]  # the node encoder reads the raw 11 features: not padded
    assert enc.shapes[0][:2] == (W, 11) and enc.out_width == W
    assert _engine.kernel_width(144) == 256  # hidden > 128: the 256-wide kernels (128 x 128 weight-gradient tiles)
    with pytest.raises(ValueError, match="at most 256"):
        _engine.kernel_width(257)


def test_data_parallel_step_refuses_to_continue_after_validation_error():
    """under data parallelism a validation error skips the optimizer update on the raising
    rank only, so the replicas diverge; the TrainStep then refuses further steps (as an exception on one
    rank ends the reference's DDP job) instead of continuing silently. Single-process steps are unaffected."""
    import pytest
    from graphphysics.training.step import TrainStep

    class _Opt:
        param_groups = []
        state = {}

    for dp, world, refuses in ((True, 2, True), (True, 1, False), (False, 1, False)):
        ts = TrainStep.__new__(TrainStep)
        ts.dp, ts.world, ts.opt, ts.sched = dp, world, _Opt(), None
        ts._raised(IndexError("edge_index out of range"))
        if refuses:
            with pytest.raises(RuntimeError, match="replicas"):
                ts._check_replicas()
        else:
            ts._check_replicas()


def test_concurrent_backward_regimes(monkeypatch):
    """conc_caps (models/_engine.py): which backward schedule each workload gets on a 256-CU device.
    Cfg B (88,560 edges, 1.8 tiles per wave): 160 + 96; Cfg E (1,395,256 edges, recomputed weight
    gradients): 128 + 128; the same graph with saved edge inputs (MGN_REW=0), small graphs and
    generic (non-chained) blocks: one stream; explicit MGN_CONC_WGRAD settings pass through."""
    from graphphysics.models import _engine as eng

    monkeypatch.setattr(eng, "_device_cus", lambda dev=None: 256)
    monkeypatch.setattr(eng, "CONC_WGRAD", "auto")
    monkeypatch.setattr(eng, "REW", "auto")
    assert eng.conc_caps(88560, True) == (160, 96)
    assert eng.conc_caps(1395256, True) == (128, 128)
    assert eng.conc_caps(11070, True) is None
    assert eng.conc_caps(88560, False) is None
    assert eng.conc_caps(1395256, False) is None
    monkeypatch.setattr(eng, "REW", "0")
    assert eng.conc_caps(1395256, True) is None
    assert eng.conc_caps(88560, True) == (160, 96)
    monkeypatch.setattr(eng, "_device_cus", lambda dev=None: 128)  # a partitioned device scales the split
    monkeypatch.setattr(eng, "REW", "auto")
    assert eng.conc_caps(1395256, True) == (64, 64)
    assert eng.conc_caps(44280, True) == (80, 48)
    monkeypatch.setattr(eng, "CONC_WGRAD", "0")
    assert eng.conc_caps(88560, True) is None
    monkeypatch.setattr(eng, "CONC_WGRAD", "168,88")
    assert eng.conc_caps(11070, False) == (168, 88)


def test_control_group_rebuilt_after_process_group_reinit(monkeypatch):
    """TrainStep's host-side control group (training/step.py control_group) is cached per rank
    set AND per default process group: after destroy_process_group() and a re-init in the same process the
    next TrainStep gets a live group, not the destroyed world's. A 1-rank gloo world posing as an RCCL one
    (get_backend patched), so the cached-gloo-group path runs on the CPU."""
    import socket

    import torch.distributed as dist
    from graphphysics.training import step as S

    def port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]

    monkeypatch.setattr(S.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(S, "_CTL_GROUPS", {})
    got = []
    for _ in range(2):
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port(), rank=0, world_size=1)
        try:
            g = S.control_group()
            assert S.control_group() is g  # cached within one world
            t = torch.ones(1)
            dist.all_reduce(t, group=g)  # usable
            got.append(g)
        finally:
            dist.destroy_process_group()
    assert got[0] is not got[1]
