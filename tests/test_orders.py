"""CPU checks of the summation-order spread the fp32 gradient parity tests use as their bound
(_orders.py): the hidden-unit permutation keeps the reference function and maps gradients back to the
original layout, and it does change the fp32 summation order."""
import torch

from oracle import mgn_oracle as O
from _orders import order_spread, relerr


def _case(mp=2, h=32, n=200, e=900, seed=3):
    g = torch.Generator().manual_seed(seed)
    ei = torch.randint(0, n, (2, e), generator=g)
    x = torch.randn(n, 11, generator=g)
    ea = torch.randn(e, 3, generator=g)
    gy = torch.randn(n, 2, generator=g)
    torch.manual_seed(0)
    rp = dict(O.OracleEPD(mp, 11, 3, 2, h).named_parameters())
    return ei, x, ea, gy, rp


def test_permuted_hidden_units_keep_the_function_and_gradients():
    ei, x, ea, gy, rp = _case()
    loss = lambda q, i=None: (O.encode_process_decode(x if i is None else i["x"], ei,  # noqa: E731
                                                      ea if i is None else i["ea"], q, 2) * gy).sum()
    loss(rp).backward()
    p64 = {k: v.detach().double().requires_grad_(True) for k, v in rp.items()}
    (O.encode_process_decode(x.double(), ei, ea.double(), p64, 2) * gy.double()).sum().backward()
    g64 = {k: v.grad for k, v in p64.items()}
    sp = order_spread(loss, rp, g64, n_orders=2,
                      inputs={"x": (x, "nodes_encoder.0.weight"), "ea": (ea, "edges_encoder.0.weight")})
    assert set(sp) == set(rp)
    # every permuted-order gradient is an fp32 evaluation of the same function: as close to fp64 as the
    # reference's own fp32 path is (shallow model, no near-ties at this size)
    for k in rp:
        assert sp[k] <= max(1e-5, 20 * relerr(rp[k].grad, g64[k])), (k, sp[k])
    assert 0.0 < max(sp.values()) < 1e-4


def test_permutation_changes_the_summation_order():
    """Not a no-op: some gradient differs bitwise from the unpermuted fp32 evaluation."""
    ei, x, ea, gy, rp = _case()
    loss = lambda q: (O.encode_process_decode(x, ei, ea, q, 2) * gy).sum()  # noqa: E731
    loss(rp).backward()
    ref = {k: v.grad.clone() for k, v in rp.items()}
    sp = order_spread(loss, rp, {k: v.double() for k, v in ref.items()}, n_orders=1)
    assert max(sp.values()) > 0.0


def test_mask_pinned_oracle_and_r8_decode():
    """Mask pinning (tests/_masks.py): the oracle on the natural ReLU branch is bitwise the reference
    ops; on a branch with one unit flipped it differs only downstream of that unit; the R8 decode
    inverts the row-octet layout of include/mgn.h mgn_mlp_saved."""
    from _masks import _r8, flips

    ei, x, ea, gy, rp = _case(mp=2, h=16)
    rec = {}
    y0 = O.encode_process_decode(x, ei, ea, rp, 2)
    y1 = O.encode_process_decode(x, ei, ea, rp, 2, masks=None, record=rec)
    masks = {k: [z > 0 for z in v] for k, v in rec.items()}
    y2 = O.encode_process_decode(x, ei, ea, rp, 2, masks=masks)
    assert torch.equal(y0, y1) and torch.equal(y0, y2)
    assert flips(masks, rec) == {}
    m2 = {k: [t.clone() for t in v] for k, v in masks.items()}
    m2["decode_module"][2][5, 3] ^= True
    f = flips(m2, rec)
    assert list(f) == ["decode_module.4"] and f["decode_module.4"]["flipped"] == 1
    y3 = O.encode_process_decode(x, ei, ea, rp, 2, masks=m2)
    assert torch.equal((y3 != y0).any(1).nonzero().flatten(), torch.tensor([5]))
    # R8: element (m, c) at ((m/8)·cols + c)·8 + m%8, rows padded to 64
    rows, cols = 70, 12
    a = torch.arange(rows * cols, dtype=torch.float32).view(rows, cols)
    buf = torch.zeros(128 * cols + 5)
    for m in range(rows):
        for c in range(cols):
            buf[5 + ((m // 8) * cols + c) * 8 + m % 8] = a[m, c]
    assert torch.equal(_r8(buf, 5, rows, cols), a)
