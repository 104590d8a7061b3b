"""North-star accuracy gate on a TRAINED model (BASELINE.json: one-step velocity MSE |Δ| ≤ 1e-5).

tests/golden/cylinder_trained.npz (tests/golden/make_golden.py gen_trained) holds what the
reference's own Simulator (MP=15, h=128, B=1, torch.manual_seed(0) init) reached after 300 training
steps on the CylinderFlow frames 0->1, 1->2, 2->3 in turn — AdamW(lr 1e-3, wd 1e-4, betas
(0.9, 0.95)) + CosineWarmupScheduler(warmup 20, max_iters 300), the reference's
lightning_module.py:111-122 training_step and configure_optimizers (275-292) — and the held-out
one-step MSE on frames 3->4 and 4->5 (eval mode, build_mask semantics, L2Loss over NORMAL ∪ OUTFLOW).

Here libmgn trains the same model from the same init the same way — the eager per-batch path the
Lightning Trainer drives (a new Batch every step), TrainStep(graph=False) — and must reach the
same held-out MSE within the reference's own run-to-run noise (bounds in the test docstring).
tests/golden/cylinder_trained_weights.npz (make_golden.py gen_trained_weights) holds the reference's
complete trained state_dict: the north-star 1e-5 gate is checked on those very weights.
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


def _train(dtype, z):
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator
    from graphphysics.training.optim import FusedAdamW
    from graphphysics.training.step import TrainStep
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data
    from graphphysics.utils.scheduler import CosineWarmupScheduler

    steps, warmup, lr = int(z["train_steps"]), int(z["warmup"]), float(z["lr"])
    torch.manual_seed(0)
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=dtype), DEV)
    for k, v in sim.state_dict().items():  # same init as the reference (RNG order)
        if ("init::" + k) in z:
            assert abs(v.double().sum().item() - float(z["init::" + k])) <= 1e-6 * (1 + abs(float(z["init::" + k])))
    opt = FusedAdamW(sim.parameters(), lr=lr, weight_decay=1e-4, betas=(0.9, 0.95))
    sch = CosineWarmupScheduler(opt, warmup=warmup, max_iters=steps)
    frames = []
    for t in range(3):
        b = meshes.cylinder_batch(1, t=t)
        frames.append(Data(**{k: torch.from_numpy(b[k]).to(DEV) for k in ("x", "y", "edge_index", "edge_attr")}))
    sts = [TrainStep(sim, opt, sch, f, graph=False) for f in frames]
    losses = torch.stack([sts[i % 3]().detach() for i in range(steps)]).cpu().numpy()
    sim.eval()
    mses = []
    for t in (3, 4):
        b = meshes.cylinder_batch(1, t=t)
        x, y = torch.from_numpy(b["x"]), torch.from_numpy(b["y"])
        d = Data(**{k: torch.from_numpy(b[k]).to(DEV) for k in ("x", "y", "edge_index", "edge_attr")})
        with torch.no_grad():
            _, _, pred = sim(d)
        pred = pred.float().cpu()
        keep = ~((x[:, 2] == 0) | (x[:, 2] == 5))
        pred[keep] = y[keep]
        mses.append(O.l2_loss(y, pred, x[:, 2]).item())
    return losses, np.array(mses), sim


HERE = os.path.join(os.path.dirname(__file__), "golden")


def _weights_fixture():
    f = os.path.join(HERE, "cylinder_trained_weights.npz")
    return np.load(f)


def _eval_frames(sim):
    """Held-out one-step MSE (frames 3->4, 4->5) and the frame-3 prediction, as the reference's
    eval_one_step (make_golden.py; lightning_module.py:168-232 build_mask semantics)."""
    from graphphysics.utils import meshes
    from graphphysics.utils.data import Data

    sim.eval()
    mses, preds = [], []
    for t in (3, 4):
        b = meshes.cylinder_batch(1, t=t)
        x, y = torch.from_numpy(b["x"]), torch.from_numpy(b["y"])
        d = Data(**{k: torch.from_numpy(b[k]).to(DEV) for k in ("x", "y", "edge_index", "edge_attr")})
        with torch.no_grad():
            _, _, pred = sim(d)
        pred = pred.float().cpu()
        keep = ~((x[:, 2] == 0) | (x[:, 2] == 5))
        pred[keep] = y[keep]
        mses.append(O.l2_loss(y, pred, x[:, 2]).item())
        preds.append(pred)
    return np.array(mses), preds


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_reference_trained_weights_one_step_mse_within_1e5(dtype):
    """The north-star gate on the REFERENCE's own trained model: the complete state_dict (weights and
    normaliser buffers, reference key names) the reference Simulator reached after 300 training steps
    (make_golden.py gen_trained_weights), loaded into the libmgn Simulator as a checkpoint, evaluated
    on the held-out frames 3->4 and 4->5: |MSE_libmgn - MSE_reference| <= 1e-5 per frame (BASELINE
    north_star), fp32 and bf16. The frame-3 prediction itself: rel-L2 <= 1e-4 (fp32) / 2e-2 (bf16)."""
    from graphphysics.models.processors import EncodeProcessDecode
    from graphphysics.models.simulator import Simulator

    z = _weights_fixture()
    sim = Simulator(11, 3, 2, 0, 2, 0, 2, 2, EncodeProcessDecode(15, 11, 3, 2, 128, compute_dtype=dtype), DEV)
    sd = {k[4:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd::")}
    missing, unexpected = sim.load_state_dict(sd, strict=True)
    assert not missing and not unexpected
    mses, preds = _eval_frames(sim)
    ref = z["one_step_mse"]
    d = np.abs(mses - ref)
    pe = float((preds[0] - torch.from_numpy(z["pred0"])).norm() / torch.from_numpy(z["pred0"]).norm())
    print(f"\n{dtype}: reference-trained weights: one-step MSE libmgn {mses} reference {ref} |d| {d}; "
          f"pred rel-L2 {pe:.2e}")
    assert np.all(d <= 1e-5), d
    assert pe <= (1e-4 if dtype == torch.float32 else 2e-2), pe


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_trained_one_step_mse_matches_reference(dtype):
    """Training is chaotic and the reference's CPU training is not even reproducible with itself:
    five runs of the same reference code from the same init (cylinder_trained.npz, and
    cylinder_trained_weights.npz chaos_* with 1, 2, 4 and 8 intra-op threads — its ATen kernels sum
    in a thread-count- and schedule-dependent order) end 300 steps at held-out MSEs up to `band` from
    their mean (the north-star 1e-5 bound holds for the same weights:
    test_reference_trained_weights_one_step_mse_within_1e5). So libmgn, training the same model from
    the same init, must (1) reproduce the first 3 steps (fp32: 1e-4 relative, before the drift;
    bf16: 2e-2), (2) end as one more draw from the reference's own run-to-run distribution:
    |MSE − mean of the reference runs| ≤ max(1e-5, 3 σ) per held-out frame, σ the runs' sample
    standard deviation (measured: runs 1.48–1.85e-4 / 2.92–3.56e-4, σ 1.5e-5 / 2.7e-5; libmgn fp32
    1.34e-4 / 2.91e-4, bf16 1.51e-4 / 2.65e-4), and (3) train as well: the median per-step
    relative distance of the loss curve from the first reference run no larger than the other
    reference runs' own (0.08–0.44: the curves decorrelate after ~5 steps, fp32 included)."""
    z = np.load(os.path.join(HERE, "cylinder_trained.npz"))
    zw = _weights_fixture()
    losses, mses, sim = _train(dtype, z)
    ref_losses = z["trained/losses"]
    runs = np.concatenate([z["trained_eval/one_step_mse"][None], zw["chaos_one_step_mse"]], 0)  # [runs, frames]
    assert runs.shape[0] >= 5
    center = runs.mean(0)
    sigma = runs.std(0, ddof=1)
    dl = np.abs(losses - ref_losses) / np.abs(ref_losses)
    print(f"\n{dtype}: one-step MSE libmgn {mses} reference runs {runs.tolist()} mean {center} sigma {sigma} "
          f"|d| {np.abs(mses - center)}; loss rel diff first 10 {np.array2string(dl[:10], precision=2)}, "
          f"median {np.median(dl):.2e}, max {dl.max():.2e}")
    fp32 = dtype == torch.float32
    np.testing.assert_allclose(losses[:3], ref_losses[:3], rtol=1e-4 if fp32 else 2e-2)
    ref_spread = max(np.median(np.abs(r - ref_losses) / np.abs(ref_losses)) for r in zw["chaos_losses"])
    assert np.median(dl) <= ref_spread, (np.median(dl), ref_spread)
    bound = np.maximum(1e-5, 3.0 * sigma)
    assert np.all(np.abs(mses - center) <= bound), (mses, center, bound)
    # normaliser accumulators after 300 training forwards: the same statistics (the means — the
    # sums of the near-zero-mean target deltas are cancellation-dominated, fp32 order-sensitive)
    for name in ("_output_normalizer", "_node_normalizer", "_edge_normalizer"):
        nrm = getattr(sim, name)
        cnt = float(z[f"trained/{name}/acc_count"])
        assert float(nrm._acc_count) == cnt
        np.testing.assert_allclose(nrm._acc_sum.cpu().double().numpy() / cnt, z[f"trained/{name}/acc_sum"] / cnt,
                                   rtol=1e-5, atol=1e-8)
        np.testing.assert_allclose(nrm._acc_sum_squared.cpu().double().numpy() / cnt,
                                   z[f"trained/{name}/acc_sum_squared"] / cnt, rtol=1e-5, atol=1e-8)
