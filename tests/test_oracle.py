"""Pin the oracle (and the product's reference-protocol host logic) to the golden vectors.

Every expected value here was produced by the REFERENCE code (tools/gen_golden.py).
"""
import numpy as np
import pytest
import torch

from conftest import golden, golden_json

from oracle import control as oc
from oracle import forward as ofw
from oracle import tables as otab

CG = golden("controllers")
CM = golden_json("controllers")
LAYERS = [tuple(x) for x in CM["layers"]]


def _eq_for(name, tok):
    if name == "main_reweight":
        return otab.equalizer_main("a dog eating a burger", "dog", (3.0,), tok)
    if name == "null_reweight_chain_refine":
        return otab.equalizer_null("a fluffy cat eating a burger", ("fluffy",), (2.0,), tok)
    if name == "null_reweight_chain_replace":
        return otab.equalizer_null("a cat eating a lasagna", ("lasagna",), (0.5,), tok)
    return None


def oracle_for(name, prompts, tok):
    steps = CM["steps"]
    if name == "main_store":
        return oc.OracleController("main", "store")
    flav = "main" if name.startswith("main") else "null"
    if name.endswith("_replace") and "chain" not in name:
        return oc.OracleController(flav, "replace", prompts, steps, {"default_": .5, "lasagna": .25}, .5, tok)
    if name.endswith("_refine") and "chain" not in name:
        return oc.OracleController(flav, "refine", prompts, steps, .75, (.25, .75), tok)
    if name == "main_reweight":
        return oc.OracleController(flav, "reweight", prompts, steps, .5, .5, tok, equalizer=_eq_for(name, tok))
    if name == "null_reweight_chain_refine":
        inner = oc.OracleController(flav, "refine", prompts, steps, .75, .5, tok)
        return oc.OracleController(flav, "reweight", prompts, steps, .75, .5, tok, equalizer=_eq_for(name, tok),
                                   inner=inner)
    if name == "null_reweight_chain_replace":
        inner = oc.OracleController(flav, "replace", prompts, steps, .5, .5, tok)
        return oc.OracleController(flav, "reweight", prompts, steps, .5, .5, tok, equalizer=_eq_for(name, tok),
                                   inner=inner)
    raise KeyError(name)


def ctrl_input(step, li):
    return torch.from_numpy(CG[f"in_s{step}_l{li}"].astype(np.float32))


@pytest.mark.parametrize("cfg", CM["configs"], ids=[c["name"] for c in CM["configs"]])
def test_oracle_controllers(cfg, tok):
    name = cfg["name"]
    ctrl = oracle_for(name, cfg["prompts"], tok)
    ctrl.num_att_layers = len(LAYERS)
    for step in range(CM["steps"]):
        for li, (place, is_cross, P, K) in enumerate(LAYERS):
            out = ctrl(ctrl_input(step, li), is_cross, place)
            want = CG[f"{name}_s{step}_l{li}"]
            assert np.array_equal(out[out.shape[0] // 2:].numpy(), want), (name, step, li)
    avg = ctrl.average()
    for key, lst in ctrl.attention_store.items():
        for i, t in enumerate(lst):
            assert np.array_equal(t.numpy(), CG[f"{name}_store_{key}_{i}"])
            assert np.array_equal(avg[key][i].numpy(), CG[f"{name}_avg_{key}_{i}"])
    assert ctrl.cur_step == int(CG[f"{name}_cur_step"])


def _product_controller(name, prompts, tok):
    from p2p_amd import controllers as pc
    from p2p_amd import null_text as pn
    steps = CM["steps"]
    cpu = torch.device("cpu")
    mod = pc if name.startswith("main") else pn
    if name == "main_store":
        return pc.AttentionStore()
    if name.endswith("_replace") and "chain" not in name:
        return mod.AttentionReplace(prompts, steps, {"default_": .5, "lasagna": .25}, .5, tokenizer=tok, device=cpu)
    if name.endswith("_refine") and "chain" not in name:
        return mod.AttentionRefine(prompts, steps, .75, (.25, .75), tokenizer=tok, device=cpu)
    if name == "main_reweight":
        eq = pc.get_equalizer(prompts[1], "dog", (3.0,), tokenizer=tok)
        return pc.AttentionReweight(prompts, steps, .5, .5, equalizer=eq, tokenizer=tok, device=cpu)
    if name == "null_reweight_chain_refine":
        eq = pn.get_equalizer(prompts[1], ("fluffy",), (2.0,), tokenizer=tok)
        inner = pn.AttentionRefine(prompts, steps, .75, .5, tokenizer=tok, device=cpu)
        return pn.AttentionReweight(prompts, steps, .75, .5, equalizer=eq, controller=inner, tokenizer=tok,
                                    device=cpu)
    if name == "null_reweight_chain_replace":
        eq = pn.get_equalizer(prompts[2], ("lasagna",), (0.5,), tokenizer=tok)
        inner = pn.AttentionReplace(prompts, steps, .5, .5, tokenizer=tok, device=cpu)
        return pn.AttentionReweight(prompts, steps, .5, .5, equalizer=eq, controller=inner, tokenizer=tok,
                                    device=cpu)
    raise KeyError(name)


@pytest.mark.parametrize("cfg", CM["configs"], ids=[c["name"] for c in CM["configs"]])
def test_product_reference_protocol(cfg, tok):
    """The product controllers' materialised-protocol methods (used for user subclasses)."""
    name = cfg["name"]
    ctrl = _product_controller(name, cfg["prompts"], tok)
    ctrl.num_att_layers = len(LAYERS)
    for step in range(CM["steps"]):
        for li, (place, is_cross, P, K) in enumerate(LAYERS):
            out = ctrl(ctrl_input(step, li), is_cross, place)
            assert np.array_equal(out[out.shape[0] // 2:].numpy(), CG[f"{name}_s{step}_l{li}"]), (name, step, li)
    for key, lst in ctrl.attention_store.items():
        for i, t in enumerate(lst):
            assert np.array_equal(t.numpy(), CG[f"{name}_store_{key}_{i}"])


# ------------------------------------------------------------------ patched forward (A1)
FG = golden("forward")
FM = golden_json("forward")


class _Attn(torch.nn.Module):
    def __init__(self, query_dim, context_dim, heads, dim_head):
        super().__init__()
        inner = heads * dim_head
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.to_q = torch.nn.Linear(query_dim, inner, bias=False)
        self.to_k = torch.nn.Linear(context_dim or query_dim, inner, bias=False)
        self.to_v = torch.nn.Linear(context_dim or query_dim, inner, bias=False)
        self.to_out = torch.nn.ModuleList([torch.nn.Linear(inner, query_dim), torch.nn.Dropout(0.0)])


_Attn.__name__ = "CrossAttention"


class _Pair(torch.nn.Module):
    def __init__(self, C, ctx, heads):
        super().__init__()
        self.attn1 = _Attn(C, None, heads, C // heads)
        self.attn2 = _Attn(C, ctx, heads, C // heads)


def forward_tree(cls_name="CrossAttention"):
    """The generator's stand-in tree, rebuilt and loaded with the fixture's weights."""
    geom = [tuple(g) for g in FM["geom"]]
    unet = torch.nn.Module()
    unet.down_blocks = torch.nn.ModuleList([_Pair(C, FM["ctx_dim"], FM["heads"]) for (pl, C, P) in geom if pl == "down"])
    unet.mid_block = _Pair(16, FM["ctx_dim"], FM["heads"])
    unet.up_blocks = torch.nn.ModuleList([_Pair(C, FM["ctx_dim"], FM["heads"]) for (pl, C, P) in geom if pl == "up"])
    sd = {k[2:]: torch.from_numpy(FG[k]) for k in FG.files if k.startswith("w_")}
    unet.load_state_dict(sd)
    model = torch.nn.Module()
    model.unet = unet
    pairs = list(unet.down_blocks) + [unet.mid_block] + list(unet.up_blocks)
    xs = [torch.from_numpy(FG[f"x{i}"]) for i in range(len(geom))]
    return model, pairs, xs, torch.from_numpy(FG["ctx"])


def test_stand_in_tree_is_named_crossattention():
    model, pairs, _, _ = forward_tree()
    assert type(pairs[0].attn1).__name__ == "CrossAttention"


def run_tree(model, pairs, xs, ctx, steps):
    outs = {}
    with torch.no_grad():
        for s in range(steps):
            for i, pair in enumerate(pairs):
                outs[(s, i, "self")] = pair.attn1(xs[i])
                outs[(s, i, "cross")] = pair.attn2(xs[i], context=ctx)
    return outs


@pytest.mark.parametrize("tag", ["dummy", "replace", "refine"])
def test_oracle_patched_forward(tag, tok):
    model, pairs, xs, ctx = forward_tree()
    steps = {"dummy": 1, "replace": 4, "refine": 3}[tag]
    if tag == "dummy":
        ctrl = None
    elif tag == "replace":
        ctrl = oc.OracleController("null", "replace", FM["prompts"], 4, {"default_": .5, "lasagna": .25}, .5, tok)
    else:
        ctrl = oc.OracleController("null", "refine", FM["refine_prompts"], 4, .75, (.25, .75), tok)
    n = ofw.install(model, ctrl)
    assert n == 2 * len(pairs)
    outs = run_tree(model, pairs, xs, ctx, steps)
    for (s, i, kind), y in outs.items():
        want = FG[f"{tag}_s{s}_p{i}_{kind}"]
        np.testing.assert_allclose(y.numpy(), want, rtol=0, atol=2e-6)
    if tag == "replace":
        assert ctrl.num_att_layers == int(FG["replace_num_att_layers"])
        for key, lst in ctrl.attention_store.items():
            for i, t in enumerate(lst):
                np.testing.assert_allclose(t.numpy(), FG[f"replace_store_{key}_{i}"], rtol=0, atol=1e-6)


# ------------------------------------------------------------------ LocalBlend (A8)
LG = golden("localblend")
LM = golden_json("localblend")


def lb_store(ci):
    store = {"down_cross": [], "up_cross": [], "mid_cross": []}
    for key in ("down_cross", "up_cross"):
        i = 0
        while f"case{ci}_{key}_{i}" in LG.files:
            store[key].append(torch.from_numpy(LG[f"case{ci}_{key}_{i}"].astype(np.float32)))
            i += 1
    return store


def lb_words(w):
    return [tuple(x) if isinstance(x, list) else x for x in w]


@pytest.mark.parametrize("ci", range(len(LM)))
def test_oracle_localblend(ci, tok):
    case = LM[ci]
    kw = dict(case["kwargs"])
    if "th" in kw:
        kw["th"] = tuple(kw["th"])
    if "substruct_words" in kw:
        kw["substruct_words"] = lb_words(kw["substruct_words"])
    lb = oc.OracleLocalBlend(case["flavour"], case["prompts"], lb_words(case["words"]), tok, **kw)
    x = torch.from_numpy(LG[f"case{ci}_x_t"])
    store = lb_store(ci)
    for c in range(case["calls"]):
        x = lb(x, store)
        assert np.array_equal(x.numpy(), LG[f"case{ci}_out{c}"])
    assert np.array_equal(tables_alpha(case, tok), LG[f"case{ci}_alpha_layers"])


def tables_alpha(case, tok):
    return otab.blend_alpha(case["prompts"], lb_words(case["words"]), tok).numpy()


# ------------------------------------------------------------------ DDIM
DG = golden("ddim")


@pytest.mark.parametrize("t", [980, 500, 20, 0])
def test_ddim_oracle_and_product(t):
    from p2p_amd.ddim import DDIMScheduler
    ac = torch.from_numpy(DG["alphas_cumprod"])
    sched = DDIMScheduler()
    sched.set_timesteps(50)
    assert torch.equal(sched.alphas_cumprod, ac)
    x, eps = torch.from_numpy(DG[f"t{t}_x"]), torch.from_numpy(DG[f"t{t}_eps"])
    assert np.array_equal(oc.ddim_prev(ac, ac[0], eps, t, x).numpy(), DG[f"t{t}_prev"])
    assert np.array_equal(oc.ddim_next(ac, ac[0], eps, t, x).numpy(), DG[f"t{t}_next"])
    assert np.array_equal(sched.prev_step(eps, t, x).numpy(), DG[f"t{t}_prev"])
    assert np.array_equal(sched.next_step(eps, t, x).numpy(), DG[f"t{t}_next"])


def test_ddim_timesteps():
    from p2p_amd.ddim import DDIMScheduler
    s = DDIMScheduler()
    s.set_timesteps(50)
    assert s.timesteps.tolist() == list(range(980, -1, -20))
