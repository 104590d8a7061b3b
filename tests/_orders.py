"""fp32 summation-order spread of the reference algorithm (test infrastructure).

A deep MLP stack has pre-activations within fp32 rounding of 0; any fp32 summation order — the
reference's ATen addmm included — may put one on either side of a ReLU, which moves the upstream
gradients by up to ~1e-3 rel-L2. Instead of a fixed tolerance for that, the parity tests measure it:
the oracle (the reference's own ops) is evaluated again in fp32 with the hidden units of every MLP
permuted (reference layers.py:77-113 `build_mlp`: Linear 0/2/4/6), the latent axis of the residual
stream permuted and the model inputs' columns permuted. The permuted model is the SAME function — unit
n of layer a and input column n of layer a+2 move together — but every layer's dot products are summed
in another k order, as libmgn's MFMA tiles sum them in yet another. The
gradients flow back through the index ops exactly (distinct indices), so each order's gradient is the
reference algorithm's fp32 gradient under a different but equally valid summation order.
"""
import torch


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _latent_perm(q, p):
    """Permute the latent feature axis of an EncodeProcessDecode parameter dict (reference
    processors.py:27-137): encoder outputs, every processor block's layer-0 input blocks and output
    rows (the residual stream), the decoder's input — the same function, every layer-0 dot product of
    the processor and the decoder (and every RMSNorm) summed in another order."""
    h = p.numel()
    for k in list(q):
        if k.endswith("_encoder.6.weight") or (k.startswith("processor_list.") and k.endswith(".6.weight")):
            q[k] = q[k][p]
        elif k.endswith(".6.bias") and not k.startswith("decode_module"):
            q[k] = q[k][p]
        elif k.endswith(".7.scale"):
            q[k] = q[k][p]
        elif k.startswith("processor_list.") and k.endswith(".0.weight"):
            nb = q[k].shape[1] // h
            q[k] = q[k][:, torch.cat([j * h + p for j in range(nb)])]
        elif k == "decode_module.0.weight":
            q[k] = q[k][:, p]


def order_spread(loss_fn, params, grads64, n_orders=3, seed=0, inputs=None):
    """Per parameter: max over `n_orders` fp32 evaluations in other summation orders of
    rel-L2(grad, fp64). Each order permutes (1) the hidden units of every MLP (Linear 0/2/4/6),
    (2) for an EncodeProcessDecode dict, the latent feature axis (`_latent_perm`), and (3) the columns
    of each model input named in `inputs` {name: (tensor, first-layer weight key)} together with that
    weight's columns. loss_fn(param_dict[, permuted_inputs]) -> scalar; grads64: the fp64
    evaluation's gradients by the same keys."""
    out = {k: 0.0 for k in params}
    g = torch.Generator().manual_seed(seed)
    prefixes = sorted({k[: -len("0.weight")] for k in params if k.endswith(".0.weight")})
    for _ in range(n_orders):
        leaves = {k: v.detach().clone().requires_grad_(True) for k, v in params.items()}
        q = dict(leaves)
        for pre in prefixes:
            for a, b in ((0, 2), (2, 4), (4, 6)):
                wa, wb = f"{pre}{a}.weight", f"{pre}{b}.weight"
                if wa not in q or wb not in q:
                    continue
                p = torch.randperm(q[wa].shape[0], generator=g)
                q[wa] = q[wa][p]
                q[f"{pre}{a}.bias"] = q[f"{pre}{a}.bias"][p]
                q[wb] = q[wb][:, p]
        if "decode_module.0.weight" in q and any(k.startswith("processor_list.") for k in q):
            _latent_perm(q, torch.randperm(q["decode_module.0.weight"].shape[1], generator=g))
        if inputs:
            ins = {}
            for name, (t, wk) in inputs.items():
                p = torch.randperm(t.shape[1], generator=g)
                ins[name] = t[:, p]
                q[wk] = q[wk][:, p]
            loss_fn(q, ins).backward()
        else:
            loss_fn(q).backward()
        for k in params:
            out[k] = max(out[k], relerr(leaves[k].grad, grads64[k]))
    return out


def assert_vs_truth_orders(got, ref32, ref64, e_order, floor=1e-5, what=""):
    """fp32 gradient parity: libmgn no further from the fp64 truth than 2x the reference's fp32 error
    for this parameter — the larger of its own path's and its worst over the permuted orders
    (`order_spread`, e_order). A near-tie flipped in block b moves the gradients of every parameter
    upstream of b by the same amount whichever summation order flips it; with 24 orders each tie that
    flips in a fair share of orders (measured: the MP=5/h=32 cylinder tie in 12 of 48) is sampled."""
    e_ref = max(relerr(ref32, ref64), e_order)
    e_got = relerr(got, ref64)
    assert e_got <= max(floor, 2 * e_ref), (
        f"{what}: libmgn {e_got:.2e} vs fp64, reference fp32 (worst summation order) {e_ref:.2e}")
