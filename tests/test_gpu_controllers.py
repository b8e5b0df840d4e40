"""Fused controller path (one HIP kernel per attention call) vs the oracle's materialised
reference semantics, over whole U-Net-shaped call sequences (GPU).

The product controller receives q, k, v exactly as the patched forward hands them over; the
oracle computes fp32 probabilities from the same q, k, applies the reference controller to
the materialised tensor and multiplies by V.
"""
import numpy as np
import pytest
import torch

from oracle import control as oc
from oracle import tables as otab
from p2p_amd import config
from p2p_amd import controllers as pc
from p2p_amd import null_text as pn

from test_gpu_kernels import ref_out, ref_probs

pytestmark = pytest.mark.gpu

# SD-v1.4 attention geometry per U-Net call: (place, P, d), self then cross
SD_LAYERS = ([("down", 4096, 40)] * 2 + [("down", 1024, 80)] * 2 + [("down", 256, 160)] * 2 +
             [("mid", 64, 160)] + [("up", 256, 160)] * 3 + [("up", 1024, 80)] * 3 + [("up", 4096, 40)] * 3)
PROMPTS = ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger",
           "a painting of a cat eating a burger", "a painting of a squirrel eating a lasagna"]
H = 8


def calls(layers):
    for place, P, d in layers:
        yield place, False, P, P, d
        yield place, True, P, 77, d


def run_pair(prod, orc, layers, steps, tol_out, tol_store, x_t=None, seed=0, qscale=1.0, prompts=None,
             io_dtype=torch.float32):
    prod.num_att_layers = orc.num_att_layers = 2 * len(layers)
    g = torch.Generator(device="cuda").manual_seed(seed)
    N = 2 * len(prompts if prompts is not None else PROMPTS)
    for step in range(steps):
        for place, is_cross, P, K, d in calls(layers):
            C = H * d
            q = (torch.randn(N, P, C, device="cuda", generator=g) * qscale).to(io_dtype)
            k = torch.randn(N, K, C, device="cuda", generator=g).to(io_dtype)
            v = torch.randn(N, K, C, device="cuda", generator=g).to(io_dtype)
            out = prod.attention(q, k, v, H, d ** -0.5, is_cross, place).float()
            probs = ref_probs(q, k, H, d ** -0.5).reshape(N * H, P, K)
            probs = orc(probs, is_cross, place)
            want = ref_out(probs.reshape(N, H, P, K), v, H)
            err = (out - want).abs().max().item()
            # the bf16 PV bound scales with the row mass of the (edited) probabilities: a reweight
            # row sums to up to max(eq), not 1 (|dO| <= 2^-7 * sum_k |p'_k| * max|V|)
            mass = max(1.0, probs.abs().sum(-1).max().item())
            assert err < tol_out * mass, (step, place, is_cross, P, err, mass)
        if x_t is not None:
            a = prod.step_callback(x_t)
            b = orc.step_callback(x_t)
            same = (a == b).all(dim=1).float().mean().item()
            assert same >= 0.999, (step, same)
            x_t = b
    assert prod.cur_step == orc.cur_step
    for key, lst in orc.attention_store.items():
        got = prod.attention_store.get(key, [])
        assert len(got) == len(lst), key
        for i, t in enumerate(lst):
            err = (got[i] - t).abs().max().item()
            assert err < tol_store, (key, i, err)


@pytest.mark.parametrize("compute", ["f32", "bf16"])
def test_replace_with_localblend_sd_geometry(cuda, tok, compute):
    words = (("squirrel", "burger"), ("lion",), ("cat",), ("lasagna",))
    steps = 3
    with config.compute_mode(compute):
        lb = pn.LocalBlend(PROMPTS, words, start_blend=0.0, tokenizer=tok, device=cuda)
        prod = pn.AttentionReplace(PROMPTS, 50, {"default_": .8, "lasagna": .3}, .4, local_blend=lb,
                                   tokenizer=tok, device=cuda)
        olb = oc.OracleLocalBlend("null", PROMPTS, words, tok, start_blend=0.0)
        orc = oc.OracleController("null", "replace", PROMPTS, 50, {"default_": .8, "lasagna": .3}, .4, tok,
                                  local_blend=olb)
        orc.mapper = orc.mapper.to(cuda)
        orc.alpha = orc.alpha.to(cuda)
        olb.alpha = olb.alpha.to(cuda)
        x_t = torch.randn(4, 4, 64, 64, device=cuda)
        tol_out = 5e-5 if compute == "f32" else 4e-2
        tol_store = 1e-5 * steps if compute == "f32" else 2e-3 * steps
        run_pair(prod, orc, SD_LAYERS, steps, tol_out, tol_store, x_t=x_t)


@pytest.mark.parametrize("flavour", ["main", "null"])
def test_refine_reweight_store_self(cuda, tok, flavour):
    prompts = ["a cat eating a burger", "a fluffy cat eating a burger", "a cat eating a burger at night",
               "a cat eating a big burger"]
    mod = pc if flavour == "main" else pn
    layers = [("down", 256, 32), ("down", 1024, 16), ("mid", 64, 32), ("up", 256, 32)]
    with config.compute_mode("f32"):
        inner = mod.AttentionRefine(prompts, 10, .5, (.1, .6), tokenizer=tok, device=cuda)
        if flavour == "main":
            eq = pc.get_equalizer(prompts[1], "fluffy", (3.0,), tokenizer=tok)
            oeq = otab.equalizer_main(prompts[1], "fluffy", (3.0,), tok)
        else:
            eq = pn.get_equalizer(prompts[1], ("fluffy", "cat"), (3.0, 0.5), tokenizer=tok)
            oeq = otab.equalizer_null(prompts[1], ("fluffy", "cat"), (3.0, 0.5), tok)
        prod = mod.AttentionReweight(prompts, 10, .5, (.1, .6), equalizer=eq, controller=inner, tokenizer=tok,
                                     device=cuda)
        oinner = oc.OracleController(flavour, "refine", prompts, 10, .5, (.1, .6), tok)
        orc = oc.OracleController(flavour, "reweight", prompts, 10, .5, (.1, .6), tok, equalizer=oeq, inner=oinner)
        for o in (oinner, orc):
            o.alpha = o.alpha.to(cuda)
        oinner.mapper = oinner.mapper.to(cuda)
        oinner.ref_alphas = oinner.ref_alphas.to(cuda)
        orc.equalizer = orc.equalizer.to(cuda)
        run_pair(prod, orc, layers, 4, 5e-5, 4e-5, qscale=3.0, prompts=prompts)


# The production edits in the production precision (bf16 MFMA kernels) at the SD geometries that
# carry them -- G1 (P 4096, d 40: cross edit only, nothing stored), G2 (P 1024, d 80) and G3 (P 256,
# d 160: self injection window, maps stored) -- at the config-2 batch (N = 8, H = 8), on peaky
# rows (q x 8 / x 16: logits std 8-16) where a bf16 error in the probabilities would show, with
# f32 inputs (split-bf16 Q.K^T, the f32-U-Net path) and bf16 inputs (the bf16 U-Net path).
# Bars (north star): stored probabilities within 2e-3 per accumulated step; O within the bf16
# PV bound 2^-7 max|V| (|V| <= ~5 here: 4e-2) -- main.py:233-278, null_text.py:290-349.
EDIT_LAYERS = [("down", 4096, 40), ("down", 1024, 80), ("down", 256, 160)]
REFINE_PROMPTS = ["a cat eating a burger", "a fluffy cat eating a burger", "a cat eating a burger at night",
                  "a cat eating a big burger"]


def _edit_pair(edit, tok, dev, steps):
    """(prompts, product controller, oracle controller) for one production edit."""
    if edit in ("refine", "reweight_refine"):
        prompts = REFINE_PROMPTS
    else:
        prompts = PROMPTS
    cross, selfw = {"default_": .8, "burger": .5}, (.0, .6)
    oalpha_spec = dict(cross)
    if edit == "refine":
        prod = pc.AttentionRefine(prompts, steps, cross, selfw, tokenizer=tok, device=dev)
        orc = oc.OracleController("main", "refine", prompts, steps, oalpha_spec, selfw, tok)
        orc.mapper, orc.ref_alphas = orc.mapper.to(dev), orc.ref_alphas.to(dev)
    else:
        eq = pc.get_equalizer(prompts[0], "burger", (2.5,), tokenizer=tok)
        oeq = otab.equalizer_main(prompts[0], "burger", (2.5,), tok).to(dev)
        inner = oinner = None
        if edit == "reweight_refine":
            inner = pc.AttentionRefine(prompts, steps, cross, selfw, tokenizer=tok, device=dev)
            oinner = oc.OracleController("main", "refine", prompts, steps, dict(cross), selfw, tok)
            oinner.mapper, oinner.ref_alphas = oinner.mapper.to(dev), oinner.ref_alphas.to(dev)
        elif edit == "reweight_replace":
            inner = pc.AttentionReplace(prompts, steps, cross, selfw, tokenizer=tok, device=dev)
            oinner = oc.OracleController("main", "replace", prompts, steps, dict(cross), selfw, tok)
            oinner.mapper = oinner.mapper.to(dev)
        if oinner is not None:
            oinner.alpha = oinner.alpha.to(dev)
        prod = pc.AttentionReweight(prompts, steps, cross, selfw, equalizer=eq, controller=inner, tokenizer=tok,
                                    device=dev)
        orc = oc.OracleController("main", "reweight", prompts, steps, oalpha_spec, selfw, tok, equalizer=oeq,
                                  inner=oinner)
    orc.alpha = orc.alpha.to(dev)
    return prompts, prod, orc


@pytest.mark.parametrize("io_dtype", [torch.float32, torch.bfloat16], ids=["f32in", "bf16in"])
@pytest.mark.parametrize("qscale", [8.0, 16.0])
@pytest.mark.parametrize("edit", ["refine", "reweight", "reweight_refine", "reweight_replace"])
def test_edits_bf16_sd_geometry(cuda, tok, edit, qscale, io_dtype):
    steps = 2
    with config.compute_mode("bf16"):
        prompts, prod, orc = _edit_pair(edit, tok, cuda, 10)
        assert prod.fused_supported()
        prog = prod._edit_program()
        # the production edit path: every weight exact in bf16 -> the dense MFMA edit (R = P0 . M)
        assert prog.dense_f16() is not None
        if edit == "refine":
            assert (prog.c_rep != 0).any()          # the c_rep * P_b term of inserted words
        if edit.startswith("reweight_"):
            assert (prog.post != 1.0).any()         # the chained post-scale
        run_pair(prod, orc, EDIT_LAYERS, steps, 4e-2, 2e-3 * steps, qscale=qscale, prompts=prompts,
                 io_dtype=io_dtype, seed=int(qscale))


def test_attention_store_only(cuda, tok):
    with config.compute_mode("f32"):
        prod = pc.AttentionStore()
        orc = oc.OracleController("main", "store")
        run_pair(prod, orc, [("down", 1024, 80), ("mid", 64, 160), ("up", 4096, 40)], 3, 5e-5, 3e-5)
        avg = prod.get_average_attention()
        oavg = orc.average()
        for key in oavg:
            for a, b in zip(avg[key], oavg[key]):
                assert (a - b).abs().max().item() < 1e-5


def test_custom_controller_materialised(cuda, tok):
    """A user subclass overriding forward gets the reference protocol on HIP-made probabilities."""
    class Halve(pc.AttentionStore):
        def forward(self, attn, is_cross, place_in_unet):
            super().forward(attn, is_cross, place_in_unet)
            return attn * 0.5

    with config.compute_mode("f32"):
        prod = Halve()
        assert not prod.fused_supported()

        class OHalve(oc.OracleController):
            def forward(self, attn, is_cross, place):
                super().forward(attn, is_cross, place)
                return attn * 0.5

        orc = OHalve("main", "store")
        run_pair(prod, orc, [("down", 256, 32), ("up", 64, 16)], 2, 5e-5, 3e-5)


def test_low_resource(cuda, tok):
    """LOW_RESOURCE: the CFG halves arrive as two calls; the first num_att_layers are skipped."""
    prompts = PROMPTS
    layers = [("down", 256, 32), ("up", 64, 32)]
    old = config.LOW_RESOURCE
    config.LOW_RESOURCE = True
    try:
        with config.compute_mode("f32"):
            prod = pn.AttentionReplace(prompts, 10, .6, .5, tokenizer=tok, device=cuda)
            orc = oc.OracleController("null", "replace", prompts, 10, .6, .5, tok, low_resource=True)
            orc.mapper, orc.alpha = orc.mapper.to(cuda), orc.alpha.to(cuda)
            prod.num_att_layers = orc.num_att_layers = 2 * len(layers)
            g = torch.Generator(device="cuda").manual_seed(1)
            B = len(prompts)
            for step in range(3):
                for half in range(2):
                    for place, is_cross, P, K, d in calls(layers):
                        C = H * d
                        q = torch.randn(B, P, C, device="cuda", generator=g)
                        k = torch.randn(B, K, C, device="cuda", generator=g)
                        v = torch.randn(B, K, C, device="cuda", generator=g)
                        out = prod.attention(q, k, v, H, d ** -0.5, is_cross, place)
                        probs = orc(ref_probs(q, k, H, d ** -0.5).reshape(B * H, P, K), is_cross, place)
                        want = ref_out(probs.reshape(B, H, P, K), v, H)
                        assert (out - want).abs().max().item() < 5e-5
            for key, lst in orc.attention_store.items():
                for i, t in enumerate(lst):
                    assert (prod.attention_store[key][i] - t).abs().max().item() < 4e-5
    finally:
        config.LOW_RESOURCE = old
