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


def run_pair(prod, orc, layers, steps, tol_out, tol_store, x_t=None, seed=0, qscale=1.0):
    prod.num_att_layers = orc.num_att_layers = 2 * len(layers)
    g = torch.Generator(device="cuda").manual_seed(seed)
    N = 2 * len(PROMPTS)
    for step in range(steps):
        for place, is_cross, P, K, d in calls(layers):
            C = H * d
            q = torch.randn(N, P, C, device="cuda", generator=g) * qscale
            k = torch.randn(N, K, C, device="cuda", generator=g)
            v = torch.randn(N, K, C, device="cuda", generator=g)
            out = prod.attention(q, k, v, H, d ** -0.5, is_cross, place)
            probs = ref_probs(q, k, H, d ** -0.5).reshape(N * H, P, K)
            probs = orc(probs, is_cross, place)
            want = ref_out(probs.reshape(N, H, P, K), v, H)
            err = (out - want).abs().max().item()
            assert err < tol_out, (step, place, is_cross, P, err)
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
        global PROMPTS
        saved = PROMPTS
        PROMPTS = prompts
        try:
            run_pair(prod, orc, layers, 4, 5e-5, 4e-5, qscale=3.0)
        finally:
            PROMPTS = saved


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
