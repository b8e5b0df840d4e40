"""The C-ABI library: builds, loads, exports every symbol include/p2p_hip.h declares, and
rejects bad arguments before launching anything (no GPU needed for these calls)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

from p2p_amd import _hip

HEADER = os.path.join(ROOT, "include", "p2p_hip.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(p2p_\w+)\s*\(", text, flags=re.M)))


def test_library_exists_and_loads():
    assert os.path.exists(_hip.library_path()), "run __graft_entry__.build()"
    L = _hip.lib()
    assert L.p2p_abi_version() == _hip.ABI_VERSION


def test_every_declared_symbol_is_exported():
    L = _hip.lib()
    names = declared_functions()
    assert len(names) >= 8
    for n in names:
        assert hasattr(L, n), n
    assert set(names) == set(_hip.EXPORTED_SYMBOLS)


def test_error_strings():
    L = _hip.lib()
    for code in (0, -1, -2, -3, -4, -5, -6):
        assert L.p2p_error_string(code)


def _tensors(**kw):
    t = _hip.AttnTensors()
    t.q = t.k = t.v = t.o = 16
    t.q_row_stride = t.k_row_stride = t.v_row_stride = t.o_row_stride = 320
    t.q_batch_stride = t.k_batch_stride = t.v_batch_stride = t.o_batch_stride = 320 * 4096
    t.n_batch, t.n_query, t.n_key, t.n_heads, t.head_dim = 8, 4096, 4096, 8, 40
    t.io_dtype, t.compute, t.scale = 0, 0, 40 ** -0.5
    for k, v in kw.items():
        setattr(t, k, v)
    return t


@pytest.mark.parametrize("kw,code", [
    (dict(q=None), -1),
    (dict(n_batch=65), -5),
    (dict(head_dim=44), -2),
    (dict(io_dtype=7), -3),
    (dict(io_dtype=1, compute=1), -3),
    (dict(q_row_stride=321), -6),
    (dict(q=8), -6),
])
def test_self_attn_rejects(kw, code):
    L = _hip.lib()
    t = _tensors(**kw)
    assert L.p2p_self_attn_fwd(ctypes.byref(t), None, None, None, 0, None, None) == code


def test_self_attn_rejects_bad_source_index():
    L = _hip.lib()
    t = _tensors()
    src = (ctypes.c_int32 * 8)(0, 1, 2, 3, 4, 5, 6, 99)
    assert L.p2p_self_attn_fwd(ctypes.byref(t), src, None, None, 0, None, None) == -5


def test_self_attn_store_needs_lse_workspace():
    # a kept map needs the row log-sum-exp scratch (rejected before any launch)
    L = _hip.lib()
    t = _tensors(n_query=1024, n_key=1024, head_dim=80)
    slots = (ctypes.c_int32 * 8)(-1, -1, -1, -1, 0, 8, 16, 24)
    assert L.p2p_self_attn_fwd(ctypes.byref(t), None, 64, slots, 1, None, None) == -1
    assert L.p2p_self_attn_fwd(ctypes.byref(t), None, 64, slots, 1, 72, None) == -6


def test_cross_attn_rejects():
    L = _hip.lib()
    t = _tensors(n_key=77)
    G = (_hip.Group * 2)()
    G[0].first, G[0].count = 0, 4
    G[1].first, G[1].count = 4, 3          # does not cover the batch
    assert L.p2p_cross_attn_fwd(ctypes.byref(t), G, 2, None, None, 0, None) == -5
    t2 = _tensors(n_key=200)
    assert L.p2p_cross_attn_fwd(ctypes.byref(t2), G, 2, None, None, 0, None) == -4
    G[1].count = 4
    G[1].program = 64                      # an edit program needs its alpha row
    assert L.p2p_cross_attn_fwd(ctypes.byref(t), G, 2, None, None, 0, None) == -1


def test_localblend_rejects():
    L = _hip.lib()
    a = _hip.BlendArgs()
    assert L.p2p_localblend(ctypes.byref(a), None) == -1
    assert L.p2p_store_scale(None, None, 1.0, 10, None) == -1


def test_clock_probe_rejects():
    L = _hip.lib()
    assert L.p2p_clock_probe(None, 8, 1000, None) == -1
    assert L.p2p_clock_probe(64, 0, 1000, None) == -1
    assert L.p2p_clock_probe(64, 8, 0, None) == -1
    assert L.p2p_clock_probe(64, 2048, 1000, None) == -1


def test_cross_attn_rejects_program_with_too_few_edits():
    """a group of 4 prompts needs a program with >= 3 edit records; one built for fewer
    would make the kernel read past the program blob and the alpha row."""
    L = _hip.lib()
    t = _tensors(n_key=77)
    G = (_hip.Group * 2)()
    G[0].first, G[0].count = 0, 4
    G[1].first, G[1].count = 4, 4
    G[1].program, G[1].alpha, G[1].n_edits = 64, 128, 2
    assert L.p2p_cross_attn_fwd(ctypes.byref(t), G, 2, None, None, 0, None) == -5


def test_library_built_from_this_tree():
    """The Makefile stamps the source hash; a stale prebuilt library fails this check."""
    from p2p_amd import _srchash
    assert _hip.lib().p2p_source_hash().decode() == _srchash.source_hash()
    assert _hip.check_source_hash() == _srchash.source_hash()


def test_production_library_ignores_variant_env(monkeypatch):
    """kernel variants are an experiments-build feature read once at load; the
    production build never reads P2P_SELF_VARIANT (its getenv is compiled out)."""
    import subprocess
    out = subprocess.run(["strings", _hip.library_path()], capture_output=True, text=True).stdout
    assert "P2P_SELF_VARIANT" not in out
