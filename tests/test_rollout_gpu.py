"""Validation rollout (reference lightning_module.py:17-25,163-249) and the inference block kernels.

test_rollout_matches_reference_fixture checks against the reference's own validation loop output
(tests/golden/rollout_golden.npz, made by tests/golden/make_golden.py gen_rollout). Tolerances: fp32 rollout vs the CPU oracle rollout (same weights, same normaliser statistics,
reference _make_prediction loop restated below): per-step predictions max|Δ| ≤ 1e-4·(1+|ref|),
rollout RMSE and per-step val losses within 1e-6 relative-ish (|Δ| ≤ 1e-6 + 1e-4·ref). Graph-replayed
rollout ≡ eager rollout bit for bit (same kernels, same order). bf16 h=128: the inference kernels
(no backward saves) produce bit-identical outputs to the training-mode kernels.
"""
import os

import numpy as np
import pytest
import torch

from oracle import mgn_oracle as O

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _built():
    import __graft_entry__ as ge

    ge.build()
    assert torch.cuda.is_available(), "GPU tests need a HIP device"


def _sim(dtype, mp, h):
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    torch.manual_seed(0)
    m = EncodeProcessDecode(mp, 11, 3, 2, h, compute_dtype=dtype)
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, m, DEV)
    # normaliser statistics from two training-mode forwards
    for t in (0, 1):
        b = meshes.cylinder_batch(2, t=t, jitter=0.01)
        with torch.no_grad():
            sim(Data(**{k: torch.from_numpy(b[k]).to(DEV) for k in ("x", "y", "edge_index", "edge_attr")}))
    sim.eval()
    return sim


def _frames(nsteps=5):
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    out = []
    for t in range(nsteps):
        b = meshes.cylinder_batch(1, t=t)
        out.append({k: torch.from_numpy(b[k]) for k in ("x", "y", "edge_index", "edge_attr")})
    return out, Data


def _oracle_rollout(sim, frames, mp, h):
    ref = O.OracleEPD(mp, 11, 3, 2, h)
    ref.load_state_dict({k: v.detach().float().cpu() for k, v in sim.model.state_dict().items()})
    osim = O.OracleSimulator(ref, 11, 3, 2)
    for mine, theirs in ((sim._output_normalizer, osim.out_norm), (sim._node_normalizer, osim.node_norm),
                         (sim._edge_normalizer, osim.edge_norm)):
        theirs.acc_sum, theirs.acc_sum_squared = mine._acc_sum.cpu(), mine._acc_sum_squared.cpu()
        theirs.acc_count, theirs.num_acc = mine._acc_count.cpu(), mine._num_accumulations.cpu()
    last, preds, losses = None, [], []
    for f in frames:  # lightning_module.py:168-202 with the batch cloned
        x, y = f["x"].clone(), f["y"]
        if last is not None:
            x[:, 0:2] = last
        nt = x[:, 2]
        mask = ~((nt == 0) | (nt == 5))
        with torch.no_grad():
            _, _, pred = osim.forward(x, y, f["edge_index"], f["edge_attr"], training=False)
        pred[mask] = y[mask]
        last = pred
        preds.append(pred)
        losses.append(O.l2_loss(y, pred, nt).item())
    p, t = torch.cat(preds), torch.cat([f["y"] for f in frames])
    return torch.stack(preds), losses, float(torch.sqrt(((p - t) ** 2).mean()))


@pytest.mark.parametrize("graph", [False, True])
def test_rollout_fp32_vs_oracle(graph):
    from graphphysics.training.rollout import Rollout

    mp, h = 5, 32
    sim = _sim(torch.float32, mp, h)
    frames, Data = _frames()
    ref, ref_losses, ref_rmse = _oracle_rollout(sim, frames, mp, h)
    ro = Rollout(sim, node_type_index=2, graph=graph)
    got = ro.rollout([Data(**{k: v.to(DEV) for k, v in f.items()}) for f in frames]).cpu()
    tol = 1e-4 * (1 + ref.abs())
    assert bool(((got - ref).abs() <= tol).all()), float((got - ref).abs().max())
    for a, b in zip([l.item() for l in ro.losses], ref_losses):
        assert abs(a - b) <= 1e-6 + 1e-4 * b
    assert abs(ro.all_rollout_rmse() - ref_rmse) <= 1e-6 + 1e-4 * ref_rmse


@pytest.mark.parametrize("graph", [False, True])
def test_rollout_matches_reference_fixture(graph):
    """Pinned to the REFERENCE's own validation loop: tests/golden/rollout_golden.npz holds what
    lightning_module.py:168-249 (validation_step over two trajectories, the reset on traj_index,
    on_validation_epoch_end's all-rollout RMSE) produced on the CylinderFlow frames with the cfgA
    model (MP=5, h=32) after 3 training steps; its full weights and normaliser buffers are loaded
    here. fp32 GPU vs the reference's CPU fp32: predictions within 1e-4·(1+|ref|), per-step
    val losses and the all-rollout RMSE within 1e-6 + 1e-4·ref."""
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.rollout import Rollout

    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "rollout_golden.npz"))
    m = EncodeProcessDecode(5, 11, 3, 2, 32, compute_dtype=torch.float32)
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, m, DEV)
    sd = {k[3:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("w::")}
    missing, unexpected = sim.load_state_dict(sd, strict=True)
    assert not missing and not unexpected
    sim.eval()
    frames, Data = _frames()
    ro = Rollout(sim, node_type_index=2, graph=graph)
    cur = 0
    for i, (traj, t) in enumerate(g["plan"].tolist()):
        if traj != cur:  # validation_step: batch.traj_index > current_val_trajectory -> reset
            ro.reset()
            cur = traj
        pred, _ = ro.step(Data(**{k: v.to(DEV) for k, v in frames[t].items()}))
        ref = torch.from_numpy(g[f"pred{i}"])
        got = pred.cpu()
        assert bool(((got - ref).abs() <= 1e-4 * (1 + ref.abs())).all()), (i, float((got - ref).abs().max()))
    for a, b in zip([l.item() for l in ro.losses], g["val_loss"].tolist()):
        assert abs(a - b) <= 1e-6 + 1e-4 * b
    ref_rmse = float(g["val_all_rollout_rmse"][0])
    assert abs(ro.all_rollout_rmse() - ref_rmse) <= 1e-6 + 1e-4 * ref_rmse


def test_rollout_graph_equals_eager_bf16_h128():
    from graphphysics.training.rollout import Rollout

    sim = _sim(torch.bfloat16, 15, 128)
    frames, Data = _frames()
    dev_frames = [Data(**{k: v.to(DEV) for k, v in f.items()}) for f in frames]
    a = Rollout(sim, 2, graph=False).rollout(dev_frames)
    b = Rollout(sim, 2, graph=True).rollout(dev_frames)
    assert torch.equal(a, b)
    # trajectory changes mesh: new edge_index tensor → re-recorded graph, still equal to eager
    from graphphysics.utils import meshes

    bb = meshes.cylinder_batch(2, t=0, jitter=0.01)
    two = [Data(**{k: torch.from_numpy(bb[k]).to(DEV) for k in ("x", "y", "edge_index", "edge_attr")})] * 3
    ro = Rollout(sim, 2, graph=True)
    ro.rollout(dev_frames)
    assert torch.equal(ro.rollout(two), Rollout(sim, 2, graph=False).rollout(two))


def test_inference_block_kernels_match_training_kernels():
    """bf16 h=128: mgn_block_forward with act = NULL (no backward saves) is bit-identical to the
    training-mode forward (same arithmetic, fewer stores)."""
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    b = meshes.cylinder_batch(8, jitter=0.01)
    g = Data(x=torch.randn(b["x"].shape[0], 11, device=DEV), edge_index=torch.from_numpy(b["edge_index"]).to(DEV),
             edge_attr=torch.from_numpy(b["edge_attr"]).to(DEV))
    torch.manual_seed(0)
    m = EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=torch.bfloat16).to(DEV)
    y_train = m(g)  # parameters require grad: training kernels with saves
    assert y_train.requires_grad
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(DEV)  # y_train's autograd graph holds the 15 blocks' saves
    torch.cuda.reset_peak_memory_stats(DEV)
    with torch.no_grad():
        y_inf = m(g)
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated(DEV) - base
    assert torch.equal(y_train.detach(), y_inf)
    # no autograd graph -> no backward saves (round 5: needs_input_grad reports requires_grad even under
    # torch.no_grad, so the grad mode is passed in): the no-grad forward's peak is one block's z / rden
    # and the residual streams, a fraction of the training forward's R8 activations, masks and z
    del y_inf
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(DEV)
    base2 = torch.cuda.memory_allocated(DEV)
    y_again = m(g)
    torch.cuda.synchronize()
    peak_train = torch.cuda.max_memory_allocated(DEV) - base2
    del y_again
    assert peak < 0.25 * peak_train, (peak, peak_train)
    from graphphysics import _native as nat

    d = m._get_plan().packed(DEV, nat.MGN_BF16).descs
    import ctypes

    # the chained bf16 h=128 block kernels have inference variants (no backward saves)
    assert nat.lib().mgn_block_forward_inference_supported(ctypes.byref(d[3]), ctypes.byref(d[4])) == 1
