"""Golden-vector generator: runs the REFERENCE's own model code (graph-physics @ /root/reference)
with two tiny stubs (tests/golden/_stubs: torch_geometric MessagePassing/Data, loguru) and writes
small .npz fixtures under tests/golden/. Run in the build container only:

    PYTHONPATH=tests/golden/_stubs:/root/reference python tests/golden/make_golden.py

What it pins:
  * GraphNetBlock fwd/bwd        reference graphphysics/models/layers.py:630-746
  * EncodeProcessDecode fwd/bwd  reference graphphysics/models/processors.py:27-137
  * Simulator train/eval         reference graphphysics/models/simulator.py:194-347
  * L2Loss                       reference graphphysics/utils/loss.py:10-65
  * AdamW + CosineWarmupScheduler reference graphphysics/training/lightning_module.py:275-292,
                                  graphphysics/utils/scheduler.py:8-67
Inputs: seeded (torch.manual_seed / numpy default_rng) and the in-tree CylinderFlow mesh
(reference tests/mock_vtu/cylinder_{0..5}.vtu, decoded by tests/golden/vtu.py and committed
as tests/golden/cylinder_mesh.npz). Weights: torch default init under manual_seed(0); the
fixture stores a per-parameter checksum so the build can prove its init consumes the RNG in
the same order, plus full weights for the small models.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
assert os.path.isdir(REF), "make_golden.py runs only where the reference is mounted"

from graphphysics.models.layers import GraphNetBlock  # noqa: E402  (reference code)
from graphphysics.models.processors import EncodeProcessDecode  # noqa: E402
from graphphysics.models.simulator import Simulator  # noqa: E402
from graphphysics.utils.loss import L2Loss  # noqa: E402
from graphphysics.utils.nodetype import NodeType  # noqa: E402
from graphphysics.utils.scheduler import CosineWarmupScheduler  # noqa: E402
from torch_geometric.data import Data  # noqa: E402  (stub)

sys.path.insert(0, HERE)
from vtu import read_vtu  # noqa: E402

torch.set_num_threads(8)
SAMPLE_ROWS = 48


def summary(prefix, t, out):
    """Store shape/sum/L2 (float64) + fixed sampled rows of a (possibly large) tensor."""
    a = t.detach().double().cpu().numpy()
    out[prefix + "__shape"] = np.array(a.shape, dtype=np.int64)
    out[prefix + "__sum"] = np.array(a.sum())
    out[prefix + "__l2"] = np.array(np.sqrt((a * a).sum()))
    if a.ndim >= 1 and a.shape[0] > 0:
        idx = np.unique(np.linspace(0, a.shape[0] - 1, SAMPLE_ROWS).astype(np.int64))
        out[prefix + "__rows_idx"] = idx
        out[prefix + "__rows"] = a[idx].astype(np.float32)


def psummary(prefix, t, out, k=32):
    """Parameter-sized summary: shape/sum/L2 + k fixed flat elements."""
    a = t.detach().double().cpu().numpy()
    out[prefix + "__shape"] = np.array(a.shape, dtype=np.int64)
    out[prefix + "__sum"] = np.array(a.sum())
    out[prefix + "__l2"] = np.array(np.sqrt((a * a).sum()))
    flat = a.reshape(-1)
    idx = np.unique(np.linspace(0, flat.size - 1, min(k, flat.size)).astype(np.int64))
    out[prefix + "__flat_idx"] = idx
    out[prefix + "__flat"] = flat[idx]


def full(prefix, t, out):
    out[prefix] = t.detach().cpu().numpy().copy()


def param_checksums(model, out, prefix="init"):
    for k, v in model.state_dict().items():
        out[f"{prefix}::{k}"] = np.array(v.double().sum().item())


# ----------------------------------------------------------------------------- mesh
def load_cylinder():
    frames = []
    for t in range(6):
        a = read_vtu(os.path.join(REF, "tests/mock_vtu", f"cylinder_{t}.vtu"))
        if t == 0:
            pos = a["Points"][:, :2].astype(np.float32)
            tri = a["connectivity"].reshape(-1, 3).astype(np.int32)
        frames.append(np.stack([a["velocity_x"], a["velocity_y"]], 1).astype(np.float32))
    vel = np.stack(frames, 0)
    return pos, tri, vel


def face_to_edge_undirected(tri, n):
    # FaceToEdge + to_undirected (coalesced => sorted by (row, col), unique)
    t = tri.astype(np.int64)
    e = np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [0, 2]]], 0)
    e = np.concatenate([e, e[:, ::-1]], 0)
    key = np.unique(e[:, 0] * n + e[:, 1])
    return np.stack([key // n, key % n], 0)


def node_types(pos, vel0):
    n = pos.shape[0]
    nt = np.full(n, int(NodeType.NORMAL), np.int64)
    inflow = pos[:, 0] == 0.0
    outflow = pos[:, 0] >= 1.6 - 1e-6
    wall = (np.linalg.norm(vel0, axis=1) == 0) & ~inflow & ~outflow
    nt[inflow] = int(NodeType.INFLOW)
    nt[outflow] = int(NodeType.OUTFLOW)
    nt[wall] = int(NodeType.WALL_BOUNDARY)
    return nt


def edge_features(pos, ei):
    # Cartesian(norm=False) + Distance(norm=False); convention chosen: pos[row] - pos[col]
    d = pos[ei[0]] - pos[ei[1]]
    return np.concatenate([d, np.linalg.norm(d, axis=1, keepdims=True)], 1).astype(np.float32)


# ----------------------------------------------------------------------------- G1
def gen_block_cycle():
    out = {}
    torch.manual_seed(0)
    # 4-node cycle made undirected (reference tests/graphphysics/models/test_layers.py:182-184)
    ei = torch.tensor([[0, 1, 1, 2, 2, 3, 3, 0], [1, 0, 2, 1, 3, 2, 0, 3]])
    key = ei[0] * 4 + ei[1]
    ei = ei[:, torch.argsort(key)]
    h = 16
    block = GraphNetBlock(hidden_size=h)
    x = torch.randn(4, h, requires_grad=True)
    e = torch.randn(8, h, requires_grad=True)
    gx = torch.randn(4, h)
    ge = torch.randn(8, h)
    x2, e2 = block(x, ei, e)
    loss = (x2 * gx).sum() + (e2 * ge).sum()
    loss.backward()
    full("edge_index", ei, out)
    full("x", x, out)
    full("e", e, out)
    full("gx", gx, out)
    full("ge", ge, out)
    full("x_out", x2, out)
    full("e_out", e2, out)
    full("x_grad", x.grad, out)
    full("e_grad", e.grad, out)
    for k, v in block.state_dict().items():
        out["w::" + k] = v.numpy().copy()
    for k, p in block.named_parameters():
        out["g::" + k] = p.grad.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "block_cycle_h16.npz"), **out)


# ----------------------------------------------------------------------------- G2
def gen_epd_random():
    out = {}
    torch.manual_seed(0)
    # reference tests/graphphysics/models/test_processors.py:9-20 (randint multigraph)
    n, ne, nin, ein, nout, h, mp = 5, 10, 8, 4, 3, 16, 3
    x = torch.randn(n, nin)
    ea = torch.randn(ne, ein)
    ei = torch.randint(0, n, (2, ne))
    model = EncodeProcessDecode(
        message_passing_num=mp, node_input_size=nin, edge_input_size=ein,
        output_size=nout, hidden_size=h,
    )
    gy = torch.randn(n, nout)
    y = model(Data(x=x, edge_index=ei, edge_attr=ea))
    (y * gy).sum().backward()
    full("x", x, out)
    full("edge_attr", ea, out)
    full("edge_index", ei, out)
    full("gy", gy, out)
    full("y", y, out)
    for k, v in model.state_dict().items():
        out["w::" + k] = v.numpy().copy()
    for k, p in model.named_parameters():
        out["g::" + k] = p.grad.numpy().copy()
    # only_processor variant on the same graph, h=16 latent inputs
    torch.manual_seed(1)
    proc = EncodeProcessDecode(
        message_passing_num=mp, node_input_size=h, edge_input_size=h,
        output_size=nout, hidden_size=h, only_processor=True,
    )
    xl = torch.randn(n, h, requires_grad=True)
    el = torch.randn(ne, h, requires_grad=True)
    gl = torch.randn(n, h)
    yl = proc(Data(x=xl, edge_index=ei, edge_attr=el))
    (yl * gl).sum().backward()
    full("op_x", xl, out)
    full("op_e", el, out)
    full("op_g", gl, out)
    full("op_y", yl, out)
    full("op_x_grad", xl.grad, out)
    full("op_e_grad", el.grad, out)
    for k, v in proc.state_dict().items():
        out["opw::" + k] = v.numpy().copy()
    for k, p in proc.named_parameters():
        out["opg::" + k] = p.grad.numpy().copy()
    np.savez_compressed(os.path.join(HERE, "epd_random_h16.npz"), **out)


# ----------------------------------------------------------------------------- cylinder
def make_sim(mp, h, seed=0):
    torch.manual_seed(seed)
    model = EncodeProcessDecode(
        message_passing_num=mp, node_input_size=2 + NodeType.SIZE, edge_input_size=3,
        output_size=2, hidden_size=h,
    )
    sim = Simulator(
        node_input_size=2 + NodeType.SIZE, edge_input_size=3, output_size=2,
        feature_index_start=0, feature_index_end=2, output_index_start=0,
        output_index_end=2, node_type_index=2, model=model, device="cpu",
    )
    return sim


def frame_data(pos, ei, ea, nt, vel, t):
    x = np.concatenate([vel[t], nt[:, None].astype(np.float32)], 1)
    return Data(
        x=torch.from_numpy(x), y=torch.from_numpy(vel[t + 1].copy()),
        pos=torch.from_numpy(pos), edge_index=torch.from_numpy(ei),
        edge_attr=torch.from_numpy(ea),
    )


def train_steps(sim, datas, out, tag, lr=1e-3, warmup=5, max_iters=100):
    loss_fn = L2Loss()
    masks = [NodeType.NORMAL, NodeType.OUTFLOW]
    opt = torch.optim.AdamW(sim.parameters(), lr=lr, weight_decay=0.0001, betas=(0.9, 0.95))
    sch = CosineWarmupScheduler(opt, warmup=warmup, max_iters=max_iters)
    sim.train()
    losses, lrs = [], []
    for i, d in enumerate(datas):
        opt.zero_grad()
        node_type = d.x[:, 2]
        net_out, tdn, _ = sim(d)
        loss = loss_fn(tdn, net_out, node_type, masks=masks)
        loss.backward()
        if i == 0:
            full(f"{tag}/step0_net_out", net_out, out)
            full(f"{tag}/step0_target_norm", tdn, out)
            for k, p in sim.named_parameters():
                psummary(f"{tag}/step0_grad::{k}", p.grad, out)
        opt.step()
        sch.step()
        losses.append(loss.item())
        lrs.append(opt.param_groups[0]["lr"])
    out[f"{tag}/losses"] = np.array(losses)
    out[f"{tag}/lrs"] = np.array(lrs)
    for k, v in sim.state_dict().items():
        psummary(f"{tag}/final::{k}", v, out)
    for name in ["_output_normalizer", "_node_normalizer", "_edge_normalizer"]:
        nrm = getattr(sim, name)
        full(f"{tag}/{name}/acc_sum", nrm._acc_sum, out)
        full(f"{tag}/{name}/acc_sum_squared", nrm._acc_sum_squared, out)
        full(f"{tag}/{name}/acc_count", nrm._acc_count, out)


def eval_one_step(sim, datas, out, tag):
    loss_fn = L2Loss()
    masks = [NodeType.NORMAL, NodeType.OUTFLOW]
    sim.eval()
    mses = []
    for i, d in enumerate(datas):
        node_type = d.x[:, 2]
        with torch.no_grad():
            _, _, pred = sim(d)
        keep = torch.logical_not((node_type == NodeType.NORMAL) | (node_type == NodeType.OUTFLOW))
        pred[keep] = d.y[keep]
        mses.append(loss_fn(d.y, pred, node_type, masks=masks).item())
        if i == 0:
            full(f"{tag}/pred0", pred, out)
    out[f"{tag}/one_step_mse"] = np.array(mses)


def gen_cylinder():
    pos, tri, vel = load_cylinder()
    n = pos.shape[0]
    ei = face_to_edge_undirected(tri, n)
    assert ei.shape[1] == 11070  # pinned by reference tests/graphphysics/dataset/test_xdmfdataset.py:173
    nt = node_types(pos, vel[0])
    ea = edge_features(pos, ei)
    np.savez_compressed(os.path.join(HERE, "cylinder_mesh.npz"), pos=pos, triangles=tri,
                        velocity=vel, node_type=nt)
    out = {}
    out["edge_index_checksum"] = np.array([ei.shape[1], int((ei[0] * 7 + ei[1] * 13).sum())])
    out["edge_attr_sum"] = np.array(ea.astype(np.float64).sum(0))

    # single h=128 block on the real mesh (latent inputs seeded)
    torch.manual_seed(0)
    h = 128
    block = GraphNetBlock(hidden_size=h)
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(n, h, generator=g).requires_grad_(True)
    e = torch.randn(ei.shape[1], h, generator=g).requires_grad_(True)
    gx = torch.randn(n, h, generator=g)
    ge = torch.randn(ei.shape[1], h, generator=g)
    x2, e2 = block(x, torch.from_numpy(ei), e)
    ((x2 * gx).sum() + (e2 * ge).sum()).backward()
    param_checksums(block, out, "blk128_init")
    summary("blk128/x_out", x2, out)
    summary("blk128/e_out", e2, out)
    summary("blk128/x_grad", x.grad, out)
    summary("blk128/e_grad", e.grad, out)
    for k, p in block.named_parameters():
        psummary(f"blk128/grad::{k}", p.grad, out)

    datas = [frame_data(pos, ei, ea, nt, vel, t) for t in range(5)]

    # Cfg A: MP=5, h=32 (training_config/cylinder.json:9-14)
    sim = make_sim(5, 32)
    param_checksums(sim, out, "cfgA_init")
    sim.eval()
    with torch.no_grad():
        y0 = sim.model(sim._build_input_graph(datas[0], is_training=False)[0])
    full("cfgA/epd_out_untrained", y0, out)
    train_steps(sim, datas[:3], out, "cfgA")
    eval_one_step(sim, datas[3:5], out, "cfgA_eval")

    # north-star model: MP=15, h=128, batch 1
    sim = make_sim(15, 128)
    param_checksums(sim, out, "cfgB_init")
    train_steps(sim, datas[:2], out, "cfgB")
    eval_one_step(sim, datas[3:5], out, "cfgB_eval")
    np.savez_compressed(os.path.join(HERE, "cylinder_golden.npz"), **out)


# ----------------------------------------------------------------------------- trained north-star model
TRAIN_STEPS, TRAIN_WARMUP, TRAIN_LR = 300, 20, 1e-3


def gen_trained():
    """North-star gate on a trained model: the reference Simulator MP=15, h=128,
    B=1, trained TRAIN_STEPS optimizer steps (frames 0->1, 1->2, 2->3 in turn; AdamW + cosine warm-up
    as lightning_module.py:275-292, scheduler.py:41-67), then the held-out one-step MSE of frames
    3->4 and 4->5 (eval mode, build_mask semantics)."""
    pos, tri, vel = load_cylinder()
    n = pos.shape[0]
    ei = face_to_edge_undirected(tri, n)
    nt = node_types(pos, vel[0])
    ea = edge_features(pos, ei)
    datas = [frame_data(pos, ei, ea, nt, vel, t) for t in range(5)]
    out = {"train_steps": np.array(TRAIN_STEPS), "warmup": np.array(TRAIN_WARMUP), "lr": np.array(TRAIN_LR)}
    sim = make_sim(15, 128)
    param_checksums(sim, out, "init")
    train_steps(sim, [datas[i % 3] for i in range(TRAIN_STEPS)], out, "trained", lr=TRAIN_LR,
                warmup=TRAIN_WARMUP, max_iters=TRAIN_STEPS)
    eval_one_step(sim, datas[3:5], out, "trained_eval")
    np.savez_compressed(os.path.join(HERE, "cylinder_trained.npz"), **out)


def gen_trained_threads1():
    """The same training run with ONE intra-op thread (a different summation order inside the
    reference's own CPU kernels): its losses and held-out MSE measure how far the reference drifts
    from itself over 300 steps, the noise floor any other implementation is compared against."""
    torch.set_num_threads(1)
    pos, tri, vel = load_cylinder()
    n = pos.shape[0]
    ei = face_to_edge_undirected(tri, n)
    nt = node_types(pos, vel[0])
    ea = edge_features(pos, ei)
    datas = [frame_data(pos, ei, ea, nt, vel, t) for t in range(5)]
    out, scratch = {}, {}
    sim = make_sim(15, 128)
    train_steps(sim, [datas[i % 3] for i in range(TRAIN_STEPS)], scratch, "trained", lr=TRAIN_LR,
                warmup=TRAIN_WARMUP, max_iters=TRAIN_STEPS)
    out["trained/losses"] = scratch["trained/losses"]
    eval_one_step(sim, datas[3:5], out, "trained_eval")
    np.savez_compressed(os.path.join(HERE, "cylinder_trained_threads1.npz"), **out)


def _train_reference(threads):
    """The gen_trained run with `threads` intra-op threads; returns (sim, losses, held-out MSEs)."""
    torch.set_num_threads(threads)
    pos, tri, vel = load_cylinder()
    n = pos.shape[0]
    ei = face_to_edge_undirected(tri, n)
    nt = node_types(pos, vel[0])
    ea = edge_features(pos, ei)
    datas = [frame_data(pos, ei, ea, nt, vel, t) for t in range(5)]
    scratch = {}
    sim = make_sim(15, 128)
    train_steps(sim, [datas[i % 3] for i in range(TRAIN_STEPS)], scratch, "trained", lr=TRAIN_LR,
                warmup=TRAIN_WARMUP, max_iters=TRAIN_STEPS)
    ev = {}
    eval_one_step(sim, datas[3:5], ev, "trained_eval")
    return sim, scratch["trained/losses"], ev["trained_eval/one_step_mse"], ev["trained_eval/pred0"]


def gen_trained_weights():
    """The reference's OWN trained model in full: gen_trained's 8-thread run
    (MP=15, h=128, 300 steps), its complete state_dict (fp32) and normaliser buffers, and its
    held-out one-step MSE / prediction — so the build evaluates the very weights the reference
    trained. Also the same run at 1, 2 and 4 threads: the reference's own run-to-run spread (its
    CPU kernels sum in thread-count-dependent order; training is chaotic), from which the
    train-from-init comparison takes its band."""
    ref = np.load(os.path.join(HERE, "cylinder_trained.npz"))
    out = {"train_steps": np.array(TRAIN_STEPS)}
    sim, losses, mse, pred0 = _train_reference(8)
    # whether this run reproduced the committed gen_trained fixture bit for bit (same code, image and
    # thread count; measured: it does not — the reference's CPU training is not reproducible with
    # itself, so the train-from-init test compares against the spread of all the runs)
    out["matches_cylinder_trained"] = np.array(bool(np.array_equal(losses, ref["trained/losses"])))
    out["losses"] = losses
    out["one_step_mse"] = mse
    out["pred0"] = pred0
    for k, v in sim.state_dict().items():
        out["sd::" + k] = v.detach().cpu().numpy().copy()
    for name in ["_output_normalizer", "_node_normalizer", "_edge_normalizer"]:
        nrm = getattr(sim, name)
        for b in ("_acc_sum", "_acc_sum_squared", "_acc_count", "_num_accumulations"):
            out[f"norm::{name}::{b}"] = getattr(nrm, b).detach().cpu().numpy().copy()
    runs = {8: (losses, mse)}
    for th in (1, 2, 4):
        _, l_t, m_t, _ = _train_reference(th)
        runs[th] = (l_t, m_t)
    out["chaos_threads"] = np.array(sorted(runs))
    out["chaos_losses"] = np.stack([runs[t][0] for t in sorted(runs)])
    out["chaos_one_step_mse"] = np.stack([runs[t][1] for t in sorted(runs)])
    torch.set_num_threads(8)
    np.savez_compressed(os.path.join(HERE, "cylinder_trained_weights.npz"), **out)


# ----------------------------------------------------------------------------- validation rollout
def _reference_lightning_module():
    """The reference LightningModule class (lightning_module.py) importable without lightning and
    the dataset / meshio stack: `lightning.LightningModule` -> nn.Module with no-op
    save_hyperparameters / log (the test captures log), and the two helper modules it imports at
    module level replaced by empty namespaces (only used by __init__ / the XDMF writer, neither of
    which the fixture calls)."""
    import types

    class _LM(torch.nn.Module):
        def save_hyperparameters(self, *a, **k):
            pass

        def log(self, name, value, **k):
            self.logged.setdefault(name, []).append(float(value))

    light = types.ModuleType("lightning")
    light.LightningModule = _LM
    sys.modules.setdefault("lightning", light)
    for name in ("graphphysics.training.parse_parameters", "graphphysics.utils.meshio_mesh"):
        mod = types.ModuleType(name)
        mod.get_model = mod.get_simulator = mod.convert_to_meshio_vtu = None
        sys.modules.setdefault(name, mod)
    from graphphysics.training.lightning_module import LightningModule

    return LightningModule


class _Batch(Data):
    def clone(self):
        return _Batch(**{k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.__dict__.items()})


def gen_rollout():
    """Reference validation rollout (lightning_module.py:168-249): validation_step over two
    trajectories (reset on traj_index change) and on_validation_epoch_end's all-rollout RMSE, with
    the cfgA model (MP=5, h=32) after 3 training steps; full weights + normaliser buffers stored."""
    pos, tri, vel = load_cylinder()
    n = pos.shape[0]
    ei = face_to_edge_undirected(tri, n)
    nt = node_types(pos, vel[0])
    ea = edge_features(pos, ei)
    datas = [frame_data(pos, ei, ea, nt, vel, t) for t in range(5)]
    sim = make_sim(5, 32)
    scratch = {}
    train_steps(sim, datas[:3], scratch, "cfgA")
    sim.eval()
    LM = _reference_lightning_module()
    lm = LM.__new__(LM)
    torch.nn.Module.__init__(lm)
    lm.logged = {}
    lm.current_epoch, lm.timestep = 0, 1.0
    lm.param = {"index": {"node_type_index": 2}}
    lm.model, lm.K, lm.loss = sim, 0, L2Loss()
    lm.loss_masks = [NodeType.NORMAL, NodeType.OUTFLOW]
    lm.use_previous_data, lm.previous_data_start, lm.previous_data_end = False, None, None
    lm.val_step_outputs, lm.val_step_targets, lm.trajectory_to_save = [], [], []
    lm.current_val_trajectory, lm.last_val_prediction, lm.last_previous_data_prediction = 0, None, None
    lm._save_trajectory_to_xdmf = lambda *a, **k: None
    lm._get_traj_savename = lambda *a, **k: ""
    out = {}
    for k, v in sim.state_dict().items():
        out["w::" + k] = v.detach().cpu().numpy().copy()
    # trajectory 0: frames 0..4 (5 predictions); trajectory 1: frames 1..3
    plan = [(0, t) for t in range(5)] + [(1, t) for t in range(1, 4)]
    for i, (traj, t) in enumerate(plan):
        d = datas[t]
        b = _Batch(x=d.x.clone(), y=d.y.clone(), pos=d.pos, edge_index=d.edge_index, edge_attr=d.edge_attr,
                   traj_index=traj)
        lm.validation_step(b, i)
        out[f"pred{i}"] = lm.val_step_outputs[-1].numpy().copy()
    out["plan"] = np.array(plan, dtype=np.int64)
    out["val_loss"] = np.array(lm.logged["val_loss"])
    lm.on_validation_epoch_end()
    out["val_all_rollout_rmse"] = np.array(lm.logged["val_all_rollout_rmse"])
    np.savez_compressed(os.path.join(HERE, "rollout_golden.npz"), **out)


if __name__ == "__main__":
    if len(sys.argv) > 1:  # e.g. make_golden.py gen_rollout gen_trained
        for name in sys.argv[1:]:
            globals()[name]()
        sys.exit(0)
    gen_block_cycle()
    gen_epd_random()
    gen_cylinder()
    gen_rollout()
    gen_trained()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
