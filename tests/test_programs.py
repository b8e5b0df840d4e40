"""Device edit programs (host side): decode the blob exactly as the cross kernel reads it and
check the result against the oracle's materialised edit (main.py:180-197 semantics)."""
import numpy as np
import pytest
import torch

from oracle import control as oc
from oracle import tables as otab
from p2p_amd import controllers as pc
from p2p_amd import null_text as pn
from p2p_amd import programs

COLS = programs.PROGRAM_COLS


def run_blob(blob: np.ndarray, P0: np.ndarray, Pb: np.ndarray, alpha: np.ndarray) -> np.ndarray:
    """Reference interpreter of the kernel's edit step (p2p_attn.hip cross_attn_kernel): every
    column walks the first tmax term planes."""
    hdr = blob[:32].view(np.int32)
    E, n, tmax = int(hdr[0]), int(hdr[1]), int(hdr[2])
    out = Pb.copy()                                   # [E, H, P, n]
    H0 = programs.HEADER_BYTES
    for e in range(E):
        rec = blob[H0 + e * programs.REC_BYTES:H0 + (e + 1) * programs.REC_BYTES]
        crep = rec[:4 * COLS].view(np.float32)
        post = rec[4 * COLS:8 * COLS].view(np.float32)
        planes = rec[8 * COLS:].view(np.int32).reshape(programs.PROGRAM_TMAX, COLS, 2)
        for w in range(n):
            pb = Pb[e, ..., w]
            acc = (crep[w] * pb).astype(np.float32)
            for t in range(tmax):
                row, val = int(planes[t, w, 0]), planes[t, w, 1:2].view(np.float32)[0]
                acc = (acc + np.float32(val) * P0[..., row]).astype(np.float32)
            R = (post[w] * acc).astype(np.float32)
            a = np.float32(alpha[e, w])
            out[e, ..., w] = (a * R + (np.float32(1) - a) * pb).astype(np.float32)
    return out


def rand_probs(shape, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * 3).softmax(-1)


PROMPTS_R = ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger",
             "a painting of a cat eating a burger", "a painting of a squirrel eating a lasagna"]
PROMPTS_F = ["a cat eating a burger", "a fluffy cat eating a burger", "a cat eating a burger at night"]


def _check(ctrl, oracle, step, tok, exact=True):
    E = ctrl.batch_size - 1
    H, P = 2, 8
    base = rand_probs((H, P, 77), 1)
    rep = rand_probs((E, H, P, 77), 2)
    alpha = ctrl.cross_replace_alpha[step].reshape(E, 77).numpy()
    got = run_blob(ctrl._edit_program().blob(), base.numpy(), rep.numpy(), alpha)
    a = oracle.alpha[step]
    want = (oracle.cross_edit(base, rep) * a + (1 - a) * rep).reshape(E, H, P, 77).numpy()
    if exact:
        assert np.array_equal(got, want)
    else:
        np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("step", [0, 30, 45])
def test_replace_program(tok, step):
    ctrl = pc.AttentionReplace(PROMPTS_R, 50, {"default_": .8, "lasagna": .2}, .4, tokenizer=tok, device="cpu")
    orc = oc.OracleController("main", "replace", PROMPTS_R, 50, {"default_": .8, "lasagna": .2}, .4, tok)
    _check(ctrl, orc, step, tok)


def test_replace_program_multitoken(tok):
    prompts = ["a beautiful mountain landscape", "a colorful mountain landscape", "pizza mountain landscape"]
    with pytest.raises(ValueError):
        pc.AttentionReplace(prompts, 10, .8, .4, tokenizer=tok, device="cpu")
    prompts = ["a beautiful mountain landscape", "a colorful mountain landscape"]
    ctrl = pc.AttentionReplace(prompts, 10, .8, .4, tokenizer=tok, device="cpu")
    orc = oc.OracleController("main", "replace", prompts, 10, .8, .4, tok)
    _check(ctrl, orc, 0, tok, exact=False)   # 3 source tokens summed per column: order may differ


@pytest.mark.parametrize("step", [0, 40])
def test_refine_program(tok, step):
    ctrl = pc.AttentionRefine(PROMPTS_F, 50, .8, .4, tokenizer=tok, device="cpu")
    orc = oc.OracleController("main", "refine", PROMPTS_F, 50, .8, .4, tok)
    _check(ctrl, orc, step, tok)


def test_reweight_programs(tok):
    eq = pc.get_equalizer(PROMPTS_F[1], "fluffy", (2.5,), tokenizer=tok)
    ctrl = pc.AttentionReweight(PROMPTS_F, 50, .8, .4, equalizer=eq, tokenizer=tok, device="cpu")
    orc = oc.OracleController("main", "reweight", PROMPTS_F, 50, .8, .4, tok, equalizer=eq)
    _check(ctrl, orc, 0, tok)
    eqn = pn.get_equalizer(PROMPTS_R[3], ("lasagna", "squirrel"), (3.0, .5), tokenizer=tok)
    inner = pn.AttentionReplace(PROMPTS_R, 50, .8, .4, tokenizer=tok, device="cpu")
    ctrl = pn.AttentionReweight(PROMPTS_R, 50, .8, .4, equalizer=eqn, controller=inner, tokenizer=tok, device="cpu")
    oinner = oc.OracleController("null", "replace", PROMPTS_R, 50, .8, .4, tok)
    orc = oc.OracleController("null", "reweight", PROMPTS_R, 50, .8, .4, tok, equalizer=eqn, inner=oinner)
    _check(ctrl, orc, 0, tok)
    inner = pn.AttentionRefine(PROMPTS_F, 50, .8, .4, tokenizer=tok, device="cpu")
    eqf = pn.get_equalizer(PROMPTS_F[1], ("fluffy",), (4.0,), tokenizer=tok)
    ctrl = pn.AttentionReweight(PROMPTS_F, 50, .8, .4, equalizer=eqf, controller=inner, tokenizer=tok, device="cpu")
    oinner = oc.OracleController("null", "refine", PROMPTS_F, 50, .8, .4, tok)
    orc = oc.OracleController("null", "reweight", PROMPTS_F, 50, .8, .4, tok, equalizer=eqf, inner=oinner)
    _check(ctrl, orc, 0, tok)


def test_fused_support_detection(tok):
    r = pc.AttentionReplace(PROMPTS_R, 50, .8, .4, tokenizer=tok, device="cpu")
    assert r.fused_supported()

    class Custom(pc.AttentionReplace):
        def replace_cross_attention(self, a, b):
            return super().replace_cross_attention(a, b) * 2

    assert not Custom(PROMPTS_R, 50, .8, .4, tokenizer=tok, device="cpu").fused_supported()

    class Blend(pn.AttentionRefine):
        def step_callback(self, x_t):   # free to override: not encoded in the kernel
            return x_t

    assert Blend(PROMPTS_F, 50, .8, .4, tokenizer=tok, device="cpu").fused_supported()

    class Inner(pc.AttentionReplace):
        def replace_cross_attention(self, a, b):
            return a
    eq = pc.get_equalizer(PROMPTS_R[1], "lion", (2.0,), tokenizer=tok)
    rw = pc.AttentionReweight(PROMPTS_R, 50, .8, .4, equalizer=eq,
                              controller=Inner(PROMPTS_R, 50, .8, .4, tokenizer=tok, device="cpu"),
                              tokenizer=tok, device="cpu")
    with pytest.raises(pc.NotFusable):
        rw._edit_program()


def test_program_blob_layout():
    m = torch.zeros(2, 77, 77)
    m[:, torch.arange(77), torch.arange(77)] = 1
    m[1, 5, 6] = 0.5                                  # column 6 of edit 1 gathers two rows
    m[1, 6, 6] = 0.5
    blob = programs.replace_program(m).blob()
    hdr = blob[:32].view(np.int32)
    dense_off = 32 + 2 * programs.REC_BYTES
    assert hdr.tolist() == [2, 77, 2, COLS, 1, dense_off, 0, 0]
    assert blob.nbytes == dense_off + 2 * 96 * 96 * 2
    planes = blob[32 + programs.REC_BYTES + 8 * COLS:dense_off].view(np.int32).reshape(8, COLS, 2)
    assert planes[0, 6].tolist() == [5, np.float32(0.5).view(np.int32)]
    assert planes[1, 6].tolist() == [6, np.float32(0.5).view(np.int32)]
    assert planes[1, 7].tolist() == [0, 0] and not planes[2:].any()
    dense = torch.from_numpy(blob[dense_off:].view(np.int16).copy()).view(torch.float16).float().reshape(2, 96, 96)
    want = torch.zeros(2, 96, 96)
    want[:, :77, :77] = m
    assert torch.equal(dense, want)


def test_program_dense_only_when_exact_in_f16():
    m = torch.zeros(1, 77, 77)
    m[0, torch.arange(77), torch.arange(77)] = 1
    m[0, 3:6, 4] = 1.0 / 3                            # 1/3 is not an f16 value
    prog = programs.replace_program(m)
    assert prog.dense_f16() is None
    blob = prog.blob()
    assert blob[:32].view(np.int32)[4:6].tolist() == [0, 0]
    assert blob.nbytes == 32 + programs.REC_BYTES


def test_program_too_many_terms_is_not_fused():
    m = torch.zeros(1, 77, 77)
    m[0, :9, 3] = 1.0 / 9
    with pytest.raises(ValueError):
        programs.replace_program(m).blob()


def test_group_batch_rejects_member_size_mismatch(tok):
    """a member built for a different prompt count than the group size (its program,
    alpha rows and LocalBlend slices are sized by it) is refused at construction."""
    import pytest
    from p2p_amd import controllers as pc
    four = ["a cat eating a burger", "a dog eating a burger", "a cow eating a burger", "a cat eating a pizza"]
    a = pc.AttentionReplace(four, 10, .8, .4, tokenizer=tok, device="cpu")
    b = pc.AttentionReplace(four[:3], 10, .8, .4, tokenizer=tok, device="cpu")
    with pytest.raises(ValueError):
        pc.GroupBatch([a, b])
    with pytest.raises(ValueError):
        pc.GroupBatch([a], group_size=3)
    c = pc.AttentionReplace(four, 10, .8, .4, tokenizer=tok, device="cpu")
    c.store_self_maps = False
    with pytest.raises(ValueError):
        pc.GroupBatch([a, c])
    assert pc.GroupBatch([a, pc.AttentionReplace(four, 10, .8, .4, tokenizer=tok, device="cpu")]).group_size == 4


def test_aggregate_attention_needs_prompt_count_for_plain_store():
    import pytest
    import torch
    from p2p_amd import controllers as pc
    store = pc.AttentionStore()
    store.attention_store = {"down_cross": [torch.rand(16, 256, 77)], "up_cross": [], "mid_cross": []}
    store.cur_step = 2
    with pytest.raises(ValueError, match="prompts="):
        pc.aggregate_attention(store, 16, ["down"], True, 0)
    out = pc.aggregate_attention(store, 16, ["down"], True, 1, prompts=["a", "b"])
    assert out.shape == (16, 16, 77)
    red = pc.reduce_maps(store, 16, ["down"], True, 2)
    assert torch.allclose(red[1], out, atol=1e-6)


def test_cross_step_plan(tok):
    """The per-step cross edit plan (AttentionControlEdit._cross_step) from the host copy of
    cross_replace_alpha (main.py:189) and the program's c_rep / post: Replace inside the window ->
    the program with GROUP_F_R_ONLY (A = 0 on every word), past cross_replace_steps -> no program
    (B = 0, A = 1: P' = P_e exactly); Refine keeps its own probabilities for the new words (A != 0)
    -> no hint; a per-word window (dict) mixes both -> the plain program."""
    from p2p_amd import _hip
    prompts = ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger"]
    rep = pc.AttentionReplace(prompts, 10, 0.8, 0.4, tokenizer=tok, device=torch.device("cpu"))
    plans = []
    for step in range(10):
        rep.cur_step = step
        prog, hints = rep._cross_step(torch.device("cpu"), 77)
        plans.append(("plain" if prog is None else "r_only" if hints == _hip.GROUP_F_R_ONLY else "edit"))
    assert plans == ["r_only"] * 8 + ["plain"] * 2, plans
    ref = pc.AttentionRefine(["a photo of a house", "a photo of a big house"], 10, 0.8, 0.4, tokenizer=tok,
                             device=torch.device("cpu"))
    ref.cur_step = 0
    prog, hints = ref._cross_step(torch.device("cpu"), 77)
    assert prog is not None and hints == 0
    ref.cur_step = 9
    assert ref._cross_step(torch.device("cpu"), 77)[0] is None
    mixed = pc.AttentionReplace(prompts, 10, {"default_": 1.0, "lion": 0.4}, 0.4, tokenizer=tok,
                                device=torch.device("cpu"))
    mixed.cur_step = 6          # "lion" past its window, every other word inside
    prog, hints = mixed._cross_step(torch.device("cpu"), 77)
    assert prog is not None and hints == 0
    # the plan follows the alpha table: an in-place change is seen at the next call
    rep.cur_step = 0
    rep.cross_replace_alpha.zero_()
    assert rep._cross_step(torch.device("cpu"), 77)[0] is None
    # a controller built under torch.inference_mode(): its alpha table has no version counter
    with torch.inference_mode():
        inf = pc.AttentionReplace(prompts, 10, 0.8, 0.4, tokenizer=tok, device=torch.device("cpu"))
        assert inf.cross_replace_alpha.is_inference()
        got = []
        for step in range(10):
            inf.cur_step = step
            prog, hints = inf._cross_step(torch.device("cpu"), 77)
            got.append(("plain" if prog is None else "r_only" if hints == _hip.GROUP_F_R_ONLY else "edit"))
    assert got == plans, got


def test_cross_kv_cache_rules():
    """ptp_utils._cross_kv: the cross-attention K / V of an unchanged context are computed once
    (ptp_utils.py:158-168 hands every step the same context); a new context object -- even with
    equal contents or at a recycled address --, an in-place change of the context, a rebuilt
    stacked weight and an inference-mode context all recompute."""
    from p2p_amd import ptp_utils as pu

    class M:
        pass
    m = M()
    g = torch.Generator().manual_seed(0)
    w = torch.randn(16, 8, generator=g)
    ctx = torch.randn(2, 5, 8, generator=g)
    calls = []
    orig = torch.nn.functional.linear

    def counting(x, weight, bias=None):
        calls.append(1)
        return orig(x, weight, bias)
    torch.nn.functional.linear = counting
    try:
        a, rows = pu._cross_kv(m, ctx, w)
        b, rows2 = pu._cross_kv(m, ctx, w)
        assert b is a and rows2 is rows and len(calls) == 1
        assert rows == (0, 1)
        assert torch.equal(a, orig(ctx, w))
        ctx.mul_(2.0)                              # in place: the version counter moves
        c, _ = pu._cross_kv(m, ctx, w)
        assert len(calls) == 2 and torch.equal(c, orig(ctx, w))
        other = ctx.clone()                        # equal contents, another tensor
        pu._cross_kv(m, other, w)
        assert len(calls) == 3
        w2 = w.clone()                             # a rebuilt stacked weight
        pu._cross_kv(m, other, w2)
        assert len(calls) == 4
        with torch.inference_mode():
            inf = torch.randn(2, 5, 8)
            pu._cross_kv(m, inf, w)
            pu._cross_kv(m, inf, w)
        assert len(calls) == 6
        pu.CACHE_CROSS_KV = False
        pu._cross_kv(m, other, w2)
        pu._cross_kv(m, other, w2)
        assert len(calls) == 8
    finally:
        torch.nn.functional.linear = orig
        pu.CACHE_CROSS_KV = True


def test_cross_kv_cache_capture_rules():
    """Under stream capture (ptp_utils._capturing, simulated here) the K / V cache keeps eager and
    captured entries apart: a capture never hits an eagerly made entry (its K / V are of the
    context's content before the replay refills it) and makes its own (the first captured step
    records the GEMM, the later captured steps reuse its output, without SHARED_KV row classes);
    an eager call never hits a captured entry (its K / V exist only after a replay)."""
    from p2p_amd import ptp_utils as pu

    class M:
        pass
    m = M()
    g = torch.Generator().manual_seed(1)
    w = torch.randn(16, 8, generator=g)
    ctx = torch.randn(2, 5, 8, generator=g)
    calls = []
    orig, orig_cap = torch.nn.functional.linear, pu._capturing
    state = {"capturing": False}

    def counting(x, weight, bias=None):
        calls.append(state["capturing"])
        return orig(x, weight, bias)
    torch.nn.functional.linear = counting
    pu._capturing = lambda t: state["capturing"]
    try:
        eager, rows = pu._cross_kv(m, ctx, w)           # eager entry (warm-up before a capture)
        assert rows == (0, 1) and calls == [False]
        state["capturing"] = True
        cap, crow = pu._cross_kv(m, ctx, w)             # capture: misses the eager entry
        assert calls == [False, True] and crow is None and cap is not eager
        cap2, _ = pu._cross_kv(m, ctx, w)               # a later captured step: hits the captured entry
        assert cap2 is cap and len(calls) == 2
        state["capturing"] = False
        again, rows2 = pu._cross_kv(m, ctx, w)          # eager: never the captured entry
        assert again is not cap and len(calls) == 3 and rows2 == (0, 1)
    finally:
        torch.nn.functional.linear = orig
        pu._capturing = orig_cap


def test_kv_row_classes_and_shared_kv_hint():
    """ptp_utils.kv_row_classes marks runs of bit-identical K / V rows (the uncond prompts "" of a
    group); _hip.shared_kv_hint turns a group whose rows all share one class into SHARED_KV."""
    from p2p_amd import _hip
    from p2p_amd import ptp_utils as pu
    g = torch.Generator().manual_seed(1)
    a, b = torch.randn(77, 16, generator=g), torch.randn(77, 16, generator=g)
    kv = torch.stack([a, a, a, a, b, a, b, b])
    rows = pu.kv_row_classes(kv)
    assert rows == (0, 0, 0, 0, 4, 5, 6, 6)
    k, v = kv[..., :8], kv[..., 8:]
    assert _hip.shared_kv_hint(k, v, 0, 4) == 0            # no row classes on the views yet
    k._p2p_rows = v._p2p_rows = rows
    assert _hip.shared_kv_hint(k, v, 0, 4) == _hip.GROUP_F_SHARED_KV
    assert _hip.shared_kv_hint(k, v, 6, 2) == _hip.GROUP_F_SHARED_KV
    assert _hip.shared_kv_hint(k, v, 4, 4) == 0             # rows 4, 5 differ
    assert _hip.shared_kv_hint(k, v, 0, 1) == 0             # one entry: nothing to share
    kv2 = kv.clone()
    kv2[2, 5, 3] += 1.0                                      # one element differs: not shared
    assert pu.kv_row_classes(kv2)[:4] == (0, 0, 2, 3)


def _tile_from_terms(blob, e):
    """The group cross kernel's mapper tile of edit e (p2p_cross.hip): zeros, then per column w the
    value of each of the first two term planes written at (row, w) where the value is non-zero."""
    hdr = blob[:32].view(np.int32)
    rec = blob[programs.HEADER_BYTES + e * programs.REC_BYTES:programs.HEADER_BYTES + (e + 1) * programs.REC_BYTES]
    planes = rec[8 * COLS:].view(np.int32).reshape(programs.PROGRAM_TMAX, COLS, 2)
    tile = np.zeros((programs.DENSE, programs.DENSE), np.float16)
    for w in range(programs.DENSE):
        for t in range(min(2, int(hdr[2]))):
            row, val = int(planes[t, w, 0]), planes[t, w, 1:2].view(np.float32)[0]
            if val != 0:
                tile[row, w] = np.float16(val)
    return tile


def test_mapper_tile_from_term_planes_equals_dense_image(tok):
    """The group cross kernel builds each edit's f16 mapper tile from the program's first two term
    planes (tmax <= 2) instead of copying the dense image: for every program kind the two tiles are
    bit-identical (Replace incl. a two-token word, Refine with -1 gathers, Reweight alone and chained
    on both, a zero equalizer entry)."""
    prompts = ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger",
               "a painting of a squirrel eating a big burger"]
    rep = pc.AttentionReplace(prompts[:2], 10, 0.8, 0.4, tokenizer=tok, device=torch.device("cpu"))
    ref = pc.AttentionRefine([prompts[0], prompts[2]], 10, 0.8, 0.4, tokenizer=tok, device=torch.device("cpu"))
    m2 = torch.zeros(1, 77, 77)
    m2[0, torch.arange(77), torch.arange(77)] = 1
    m2[0, 3:5, 4] = 0.5                                # a target word fed by two source words (tmax 2)
    eq = torch.rand(1, 77, generator=torch.Generator().manual_seed(3)).half().float()   # (dense: f16-exact)
    eq[0, 5] = 0.0
    progs = [rep._edit_program(), ref._edit_program(), programs.replace_program(m2),
             programs.reweight_program(eq, 1, None), programs.reweight_program(eq, 1, rep._edit_program()),
             programs.reweight_program(eq, 1, ref._edit_program())]
    for prog in progs:
        blob = prog.blob()
        hdr = blob[:32].view(np.int32)
        assert hdr[4] == 1 and hdr[2] <= 2
        dense = blob[int(hdr[5]):].view(np.float16).reshape(prog.n_edits, programs.DENSE, programs.DENSE)
        for e in range(prog.n_edits):
            assert np.array_equal(_tile_from_terms(blob, e).view(np.uint16), dense[e].view(np.uint16))
