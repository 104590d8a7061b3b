"""C-ABI checks (CPU only, no kernel launches): the library loads, exports exactly what
include/mgn.h declares, the ctypes mirrors match the C struct layouts, and the pure host-side
size functions agree with the layout rules the kernels use."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "mgn.h")


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as ge

    ge.build()
    from graphphysics import _native as nat

    return nat.load()


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(mgn_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_and_library_exports_every_symbol(lib):
    from graphphysics import _native as nat

    decl = header_functions()
    assert len(decl) >= 20
    assert sorted(nat.EXPORTS) == decl, set(decl) ^ set(nat.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (mgn_\w+)", out))
    assert set(decl) <= exported, set(decl) - exported
    for name in decl:
        assert getattr(lib, name) is not None


def test_ctypes_struct_layouts_match_c(lib):
    from graphphysics import _native as nat

    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "mgn.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("mgn_topology %zu\n", sizeof(mgn_topology));
  printf("mgn_mlp %zu\n", sizeof(mgn_mlp));
  printf("mgn_mlp_saved %zu\n", sizeof(mgn_mlp_saved));
  printf("mgn_block_saved %zu\n", sizeof(mgn_block_saved));
  printf("mgn_pack_job %zu\n", sizeof(mgn_pack_job));
  P(mgn_topology, row_perm) P(mgn_mlp, wpack) P(mgn_mlp, bias) P(mgn_mlp, scale)
  P(mgn_mlp_saved, rden) P(mgn_block_saved, node) P(mgn_block_saved, aggr) P(mgn_pack_job, n)
  P(mgn_mlp, norm_dim) P(mgn_pack_job, n_src) P(mgn_pack_job, kb_pad) P(mgn_block_saved, proj)
  printf("mgn_wgrad_reduce %zu\n", sizeof(mgn_wgrad_reduce));
  P(mgn_wgrad_reduce, nchunks_x) P(mgn_wgrad_reduce, hoff) P(mgn_wgrad_reduce, nchunks_h)
  printf("mgn_call_opts %zu\n", sizeof(mgn_call_opts));
  P(mgn_call_opts, wgrad_cus) P(mgn_call_opts, err_word)
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "probe.c")
        open(c, "w").write(probe)
        exe = os.path.join(d, "probe")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(line.rsplit(" ", 1) for line in lines if line)
    assert int(got["mgn_topology"]) == ctypes.sizeof(nat.Topology)
    assert int(got["mgn_mlp"]) == ctypes.sizeof(nat.Mlp)
    assert int(got["mgn_mlp_saved"]) == ctypes.sizeof(nat.MlpSaved)
    assert int(got["mgn_block_saved"]) == ctypes.sizeof(nat.BlockSaved)
    assert int(got["mgn_pack_job"]) == ctypes.sizeof(nat.PackJob)
    assert int(got["mgn_topology.row_perm"]) == nat.Topology.row_perm.offset
    assert int(got["mgn_mlp.wpack"]) == nat.Mlp.wpack.offset
    assert int(got["mgn_mlp.bias"]) == nat.Mlp.bias.offset
    assert int(got["mgn_mlp.scale"]) == nat.Mlp.scale.offset
    assert int(got["mgn_mlp_saved.rden"]) == nat.MlpSaved.rden.offset
    assert int(got["mgn_block_saved.node"]) == nat.BlockSaved.node.offset
    assert int(got["mgn_block_saved.aggr"]) == nat.BlockSaved.aggr.offset
    assert int(got["mgn_pack_job.n"]) == nat.PackJob.n.offset
    assert int(got["mgn_mlp.norm_dim"]) == nat.Mlp.norm_dim.offset
    assert int(got["mgn_pack_job.n_src"]) == nat.PackJob.n_src.offset
    assert int(got["mgn_pack_job.kb_pad"]) == nat.PackJob.kb_pad.offset
    assert int(got["mgn_block_saved.proj"]) == nat.BlockSaved.proj.offset
    assert int(got["mgn_wgrad_reduce"]) == ctypes.sizeof(nat.WgradReduce)
    for f in ("nchunks_x", "hoff", "nchunks_h"):
        assert int(got["mgn_wgrad_reduce." + f]) == getattr(nat.WgradReduce, f).offset
    assert int(got["mgn_call_opts"]) == ctypes.sizeof(nat.CallOpts)
    for f in ("wgrad_cus", "err_word"):
        assert int(got["mgn_call_opts." + f]) == getattr(nat.CallOpts, f).offset


def test_host_size_functions(lib):
    from graphphysics import _native as nat

    assert lib.mgn_abi_version() == 17
    # fragment-packed Linear: max(fwd, transposed) fragment count x 64 lanes x VEC
    assert lib.mgn_linear_pack_elems(128, 384, nat.MGN_BF16) == max(8 * 12, 24 * 4) * 64 * 8
    assert lib.mgn_linear_pack_elems(2, 128, nat.MGN_F32) == max(1 * 32, 8 * 1) * 64
    # fp32 128-wide Linears also carry a 128x128 chain image per 128-column block (fp32 chained kernels)
    assert lib.mgn_linear_pack_elems(128, 384, nat.MGN_F32) == max(8 * 96, 24 * 32) * 64 + 3 * 128 * 128
    assert lib.mgn_linear_pack_elems(128, 100, nat.MGN_F32) == max(8 * 25, 8 * 32) * 64
    m = nat.Mlp()
    m.n_layers, m.in_dim, m.hidden, m.out_dim, m.has_norm, m.dtype = 4, 384, 128, 128, 1, nat.MGN_BF16
    ae, mw = ctypes.c_int64(), ctypes.c_int64()
    assert lib.mgn_mlp_saved_elems(ctypes.byref(m), 1000, 0, ctypes.byref(ae), ctypes.byref(mw)) == 0
    rp = 1024  # rows padded to 64
    assert ae.value == rp * (384 + 3 * 128)
    assert mw.value == 3 * (rp // 16) * (128 // 16) * 4
    assert lib.mgn_mlp_saved_elems(ctypes.byref(m), 1000, 1, ctypes.byref(ae), ctypes.byref(mw)) == 0
    assert ae.value == rp * 3 * 128  # GraphNetBlock MLPs re-gather their layer-0 input
    assert lib.mgn_mlp_backward_workspace_bytes(ctypes.byref(m), 1000) > 4 * rp * 128 * 2


def test_errors_without_device_are_reported_not_crashing(lib):
    from graphphysics import _native as nat

    m = nat.Mlp()
    m.n_layers, m.in_dim, m.hidden, m.out_dim, m.has_norm, m.dtype = 1, 8, 128, 128, 1, nat.MGN_BF16
    s = nat.MlpSaved()
    rc = lib.mgn_mlp_forward(ctypes.byref(m), None, 0, 8, None, 10, None, 0, ctypes.byref(s), None)
    assert rc != 0
    assert b"at least 2 layers" in lib.mgn_last_error()


def test_no_process_global_launch_state(lib):
    """ABI v17: the CU caps are per-call arguments (mgn_call_opts), so the header
    declares no setter of library-wide state and says so; a negative cap is rejected by the call itself
    (before any device work)."""
    from graphphysics import _native as nat

    decl = header_functions()
    assert "mgn_set_grid_cus" not in decl and not any(n.startswith("mgn_set_") for n in decl)
    src = open(HEADER).read()
    assert "no global mutable state besides the" in src and "mgn_call_opts" in src
    m = nat.Mlp()
    m.n_layers, m.in_dim, m.hidden, m.out_dim, m.has_norm, m.dtype = 4, 8, 128, 128, 1, nat.MGN_BF16
    bad = nat.CallOpts(-1, 0, None)
    rc = lib.mgn_mlp_backward_deferred3(ctypes.byref(m), None, 0, 8, None, 10, None, None, 0, None, 0, None, None,
                                        0, None, 0, ctypes.byref(nat.WgradReduce()), 0, ctypes.byref(bad), None)
    assert rc != 0 and b"CU caps" in lib.mgn_last_error()
    t = nat.Topology()
    rc = lib.mgn_block_backward_deferred3(ctypes.byref(t), ctypes.byref(m), ctypes.byref(m), None, None, None, None,
                                          None, None, None, None, None, None, 0, None, 0,
                                          (nat.WgradReduce * 2)(), 0, ctypes.byref(nat.CallOpts(0, -4, None)), None)
    assert rc != 0 and b"CU caps" in lib.mgn_last_error()
