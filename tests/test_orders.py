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
