#!/usr/bin/env python
"""Generate golden vectors by RUNNING THE REFERENCE in this container.

TEST INFRASTRUCTURE ONLY.  Refuses to run unless /root/reference exists.  Writes small
``.npz``/``.json`` fixtures into ``tests/golden``; the reference code itself is never
copied (it is imported / AST-loaded in place by ``tools/refload.py``).

Fixtures (all inputs are stored with the outputs, ids included):

* ``tables.npz``      A9: replacement / refinement mappers, word indices, time-word
                       alphas (float / tuple / dict forms), equalizers (main + null_text).
* ``controllers.npz`` A2-A7: the reference controllers' outputs for a multi-step sequence of
                       synthetic softmax tensors, plus the final AttentionStore contents.
* ``forward.npz``     A1: the reference ``register_attention_control`` patched forward on an
                       SD-shaped stand-in module tree with seeded weights, over 4 steps.
* ``localblend.npz``  A8: LocalBlend (main form B=2; null_text form B=2/4, substruct,
                       start_blend gating) masks applied to latents.
* ``ddim.npz``        DDIM prev/next step restated in ``null_text.py:471-489``.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "prompt-to-prompt_amd"))

if not os.path.isdir("/root/reference"):
    raise SystemExit("gen_golden.py needs /root/reference (build container only)")

from refload import load_ref_modules, load_script_classes  # noqa: E402
from p2p_amd.tokenizer import StandInTokenizer  # noqa: E402

TOK = StandInTokenizer()
ref_ptp, ref_sa = load_ref_modules()

# --------------------------------------------------------------------------- prompts
REPLACE_SETS = [
    ["a cat sitting on a car", "a dog sitting on a car"],
    ["a photo of a burger", "a photo of a lasagna"],                       # 1 -> 2 tokens
    ["a squirrel eating a burger", "a lion eating a burger"],              # 2 -> 1 tokens
    ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger",
     "a painting of a cat eating a burger", "a painting of a squirrel eating a lasagna"],
    ["people walks in the city at bright afternoon", "people walks in the city at dark night"],
    ["a cat and a cat", "a dog and a cat"],
    ["a beautiful mountain landscape", "a colorful mountain landscape"],   # 3 -> 2 tokens
    ["pizza on a table", "spaghetti on a table"],                          # 1 -> 3 tokens
    ["a red bicycle near a lake", "a blue bicycle near a lake", "a red motorcycle near a lake",
     "a red bicycle near a waterfall"],
    ["a house", "a castle"],
    ["an astronaut riding a horse", "an astronaut riding a dragon", "an astronaut riding a unicorn"],
    ["a big dog", "a big dog"],                                            # no change
]
REFINE_SETS = [
    ["a castle next to a river", "children drawing of a castle next to a river"],
    ["a cat", "a fluffy cat", "a cat wearing sunglasses"],
    ["a photo of a house on a mountain", "a photo of a house on a mountain at winter",
     "a watercolor photo of a house on a mountain"],
    ["a big red car", "a car"],
    ["a squirrel eating a burger", "a squirrel eating a huge lasagna burger"],
    ["a painting of a squirrel eating a burger", "a realistic painting of a squirrel eating a burger",
     "a painting of a squirrel eating a burger in the snow",
     "a painting of a squirrel eating a delicious burger"],
]
WORD_QUERIES = [
    ("a painting of a squirrel eating a burger", "squirrel"),
    ("a painting of a squirrel eating a burger", "burger"),
    ("a painting of a squirrel eating a burger", 4),
    ("a painting of a squirrel eating a burger", "a"),
    ("a photo of a lasagna", "lasagna"),
    ("people walks in the city at bright afternoon", "afternoon"),
    ("people walks in the city at bright afternoon", "night"),
    ("a beautiful mountain landscape", "beautiful"),
    ("a beautiful mountain landscape", 3),
    ("spaghetti on a table", "spaghetti"),
]
ALPHA_FORMS = [
    ("f0.8", 0.8),
    ("t0.2_0.6", (0.2, 0.6)),
    ("d_default1_lasagna0.2", {"default_": 1., "lasagna": 0.2}),
    ("d_default0_0.5_cat0.3_0.9", {"default_": (0., 0.5), "cat": (0.3, 0.9)}),
    ("d_burger0.4", {"burger": 0.4}),
    ("f0.0", 0.0),
    ("f1.0", 1.0),
]
ALPHA_PROMPTS = [
    ["a photo of a cat eating a burger", "a photo of a dog eating a lasagna",
     "a photo of a cat eating a burger at night"],
    ["a cat sitting on a car", "a dog sitting on a car"],
]


def _t(x):
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def gen_tables():
    main_ns = load_script_classes("main.py", TOK)
    nt_ns = load_script_classes("null_text.py", TOK,
                                extra_globals={"x_t": torch.zeros(1, 4, 64, 64)})
    out, manifest = {}, {"replace": [], "refine": [], "words": [], "alphas": [], "eq_main": [],
                         "eq_null": []}
    for i, prompts in enumerate(REPLACE_SETS):
        out[f"replace{i}"] = _t(ref_sa.get_replacement_mapper(prompts, TOK))
        manifest["replace"].append({"prompts": prompts, "ids": [TOK.encode(p) for p in prompts]})
    for i, prompts in enumerate(REFINE_SETS + REPLACE_SETS):
        m, a = ref_sa.get_refinement_mapper(prompts, TOK)
        out[f"refine{i}_mapper"] = _t(m)
        out[f"refine{i}_alphas"] = _t(a)
        manifest["refine"].append({"prompts": prompts, "ids": [TOK.encode(p) for p in prompts]})
    for i, (text, w) in enumerate(WORD_QUERIES):
        out[f"words{i}"] = _t(ref_ptp.get_word_inds(text, w, TOK)).astype(np.int64)
        out[f"words{i}_sa"] = _t(ref_sa.get_word_inds(text, w, TOK)).astype(np.int64)
        manifest["words"].append({"text": text, "word": w})
    for pi, prompts in enumerate(ALPHA_PROMPTS):
        for name, form in ALPHA_FORMS:
            for n in (50, 7):
                arg = dict(form) if isinstance(form, dict) else form
                a = ref_ptp.get_time_words_attention_alpha(prompts, n, arg, TOK)
                key = f"alpha{pi}_{name}_n{n}"
                out[key] = _t(a)
                manifest["alphas"].append({"key": key, "prompts": prompts, "form": form,
                                           "num_steps": n})
    eq_main = [("a cat sitting on a car", "cat", (2.0,)),
               ("a cat sitting on a car", ("cat", "car"), (3.0,)),
               ("a cat sitting on a car", 1, (0.5,)),
               ("a photo of a lasagna", "lasagna", (4.0,)),
               ("a photo of a lasagna", "lasagna", (4.0, -2.0))]   # #tokens == #values
    for i, (text, ws, vals) in enumerate(eq_main):
        out[f"eq_main{i}"] = _t(main_ns["get_equalizer"](text, ws, vals))
        manifest["eq_main"].append({"text": text, "words": ws, "values": vals})
    eq_null = [("a cat sitting on a car", ("cat", "car"), (2.0, -1.0)),
               ("a photo of a lasagna", ("lasagna",), (5.0,)),
               ("a photo of a burger", "burger", (0.0,)),
               ("a painting of a squirrel eating a burger", (4, "burger"), (2.5, 0.25))]
    for i, (text, ws, vals) in enumerate(eq_null):
        out[f"eq_null{i}"] = _t(nt_ns["get_equalizer"](text, ws, vals))
        manifest["eq_null"].append({"text": text, "words": ws, "values": vals})
    np.savez_compressed(os.path.join(OUT, "tables.npz"), **out)
    with open(os.path.join(OUT, "tables.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("tables:", len(out), "arrays")


# --------------------------------------------------------------------------- controllers
# (place, is_cross, P, K): every geometry class the controllers distinguish.
CTRL_LAYERS = [("down", False, 16, 16), ("down", True, 16, 77),
               ("down", False, 4, 512), ("down", True, 4, 77),
               ("mid", False, 8, 8), ("mid", True, 8, 77),
               ("up", False, 16, 16), ("up", True, 16, 77)]
CTRL_PROMPTS_REPLACE = ["a cat eating a burger", "a dog eating a burger", "a cat eating a lasagna"]
CTRL_PROMPTS_REFINE = ["a cat eating a burger", "a fluffy cat eating a burger",
                       "a cat eating a burger at night"]
CTRL_H = 2
CTRL_STEPS = 4


def _fp16_exact(x):
    return x.half().float()


def _ctrl_inputs(B):
    g = torch.Generator().manual_seed(1234)
    inputs = []
    for step in range(CTRL_STEPS):
        per = []
        for (place, is_cross, P, K) in CTRL_LAYERS:
            logits = torch.randn(2 * B * CTRL_H, P, K, generator=g) * 3.0
            per.append(_fp16_exact(logits.softmax(-1)))
        inputs.append(per)
    return inputs


def _ctrl_configs(main_ns, nt_ns):
    B = 3
    cfgs = []
    for flav, ns in (("main", main_ns), ("null", nt_ns)):
        cfgs.append((f"{flav}_replace", CTRL_PROMPTS_REPLACE,
                     lambda ns=ns: ns["AttentionReplace"](CTRL_PROMPTS_REPLACE, CTRL_STEPS,
                                                          cross_replace_steps={"default_": .5, "lasagna": .25},
                                                          self_replace_steps=.5)))
        cfgs.append((f"{flav}_refine", CTRL_PROMPTS_REFINE,
                     lambda ns=ns: ns["AttentionRefine"](CTRL_PROMPTS_REFINE, CTRL_STEPS,
                                                         cross_replace_steps=.75,
                                                         self_replace_steps=(.25, .75))))
    eq = main_ns["get_equalizer"](CTRL_PROMPTS_REPLACE[1], "dog", (3.0,))
    cfgs.append(("main_reweight", CTRL_PROMPTS_REPLACE,
                 lambda: main_ns["AttentionReweight"](CTRL_PROMPTS_REPLACE, CTRL_STEPS, .5, .5,
                                                      equalizer=eq)))
    eqn = nt_ns["get_equalizer"](CTRL_PROMPTS_REFINE[1], ("fluffy",), (2.0,))
    cfgs.append(("null_reweight_chain_refine", CTRL_PROMPTS_REFINE,
                 lambda: nt_ns["AttentionReweight"](
                     CTRL_PROMPTS_REFINE, CTRL_STEPS, .75, .5, equalizer=eqn,
                     controller=nt_ns["AttentionRefine"](CTRL_PROMPTS_REFINE, CTRL_STEPS, .75, .5))))
    eqr = nt_ns["get_equalizer"](CTRL_PROMPTS_REPLACE[2], ("lasagna",), (0.5,))
    cfgs.append(("null_reweight_chain_replace", CTRL_PROMPTS_REPLACE,
                 lambda: nt_ns["AttentionReweight"](
                     CTRL_PROMPTS_REPLACE, CTRL_STEPS, .5, .5, equalizer=eqr,
                     controller=nt_ns["AttentionReplace"](CTRL_PROMPTS_REPLACE, CTRL_STEPS, .5, .5))))
    cfgs.append(("main_store", CTRL_PROMPTS_REPLACE, lambda: main_ns["AttentionStore"]()))
    return B, cfgs


def gen_controllers():
    main_ns = load_script_classes("main.py", TOK)
    nt_ns = load_script_classes("null_text.py", TOK,
                                extra_globals={"x_t": torch.zeros(1, 4, 64, 64)})
    B, cfgs = _ctrl_configs(main_ns, nt_ns)
    inputs = _ctrl_inputs(B)
    out = {}
    for step in range(CTRL_STEPS):
        for li in range(len(CTRL_LAYERS)):
            out[f"in_s{step}_l{li}"] = inputs[step][li].half().numpy()
    names = []
    for name, prompts, make in cfgs:
        ctrl = make()
        ctrl.num_att_layers = len(CTRL_LAYERS)
        for step in range(CTRL_STEPS):
            for li, (place, is_cross, P, K) in enumerate(CTRL_LAYERS):
                attn = inputs[step][li].clone()
                res = ctrl(attn, is_cross, place)
                half = res.shape[0] // 2
                # copy: the store keeps aliasing views that later steps add into
                out[f"{name}_s{step}_l{li}"] = res[half:].numpy().copy()
                # the uncond half must come back untouched
                assert torch.equal(res[:half], inputs[step][li][:half])
        avg = ctrl.get_average_attention()
        for key, lst in ctrl.attention_store.items():
            for i, t in enumerate(lst):
                out[f"{name}_store_{key}_{i}"] = t.numpy()
                out[f"{name}_avg_{key}_{i}"] = avg[key][i].numpy()
        out[f"{name}_cur_step"] = np.array(ctrl.cur_step)
        names.append({"name": name, "prompts": prompts,
                      "ids": [TOK.encode(p) for p in prompts]})
    np.savez_compressed(os.path.join(OUT, "controllers.npz"), **out)
    with open(os.path.join(OUT, "controllers.json"), "w") as f:
        json.dump({"configs": names, "layers": CTRL_LAYERS, "heads": CTRL_H,
                   "steps": CTRL_STEPS, "batch": B}, f, indent=1)
    print("controllers:", len(out), "arrays")


# --------------------------------------------------------------------------- patched forward
class CrossAttention(torch.nn.Module):
    """Stand-in with the diffusers-0.8.1 attribute surface the hook uses."""

    def __init__(self, query_dim, context_dim=None, heads=2, dim_head=16):
        super().__init__()
        inner = heads * dim_head
        context_dim = context_dim or query_dim
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.to_q = torch.nn.Linear(query_dim, inner, bias=False)
        self.to_k = torch.nn.Linear(context_dim, inner, bias=False)
        self.to_v = torch.nn.Linear(context_dim, inner, bias=False)
        self.to_out = torch.nn.ModuleList([torch.nn.Linear(inner, query_dim), torch.nn.Dropout(0.0)])

    def reshape_heads_to_batch_dim(self, t):
        b, s, dim = t.shape
        h = self.heads
        return t.reshape(b, s, h, dim // h).permute(0, 2, 1, 3).reshape(b * h, s, dim // h)

    def reshape_batch_dim_to_heads(self, t):
        bh, s, d = t.shape
        h = self.heads
        return t.reshape(bh // h, h, s, d).permute(0, 2, 1, 3).reshape(bh // h, s, d * h)


class _Pair(torch.nn.Module):
    def __init__(self, C, ctx_dim, heads):
        super().__init__()
        self.attn1 = CrossAttention(C, None, heads, C // heads)
        self.attn2 = CrossAttention(C, ctx_dim, heads, C // heads)


FWD_GEOM = [("down", 32, 64), ("down", 16, 64), ("mid", 16, 4), ("up", 32, 64), ("up", 32, 16)]
FWD_PROMPTS = ["a cat eating a burger", "a dog eating a burger", "a cat eating a lasagna"]


def _fwd_tree(ctx_dim=24, heads=2):
    torch.manual_seed(7)
    unet = torch.nn.Module()
    unet.down_blocks = torch.nn.ModuleList([_Pair(C, ctx_dim, heads) for (pl, C, P) in FWD_GEOM if pl == "down"])
    unet.mid_block = _Pair(16, ctx_dim, heads)
    unet.up_blocks = torch.nn.ModuleList([_Pair(C, ctx_dim, heads) for (pl, C, P) in FWD_GEOM if pl == "up"])
    model = torch.nn.Module()
    model.unet = unet
    pairs = list(unet.down_blocks) + [unet.mid_block] + list(unet.up_blocks)
    return model, pairs


def gen_forward():
    nt_ns = load_script_classes("null_text.py", TOK,
                                extra_globals={"x_t": torch.zeros(1, 4, 64, 64)})
    B = len(FWD_PROMPTS)
    out = {}
    model, pairs = _fwd_tree()
    for name, p in model.unet.named_parameters():
        out["w_" + name] = p.detach().numpy()
    g = torch.Generator().manual_seed(99)
    xs = [torch.randn(2 * B, P, C, generator=g) for (pl, C, P) in FWD_GEOM]
    ctx = torch.randn(2 * B, 77, 24, generator=g)
    for i, x in enumerate(xs):
        out[f"x{i}"] = x.numpy()
    out["ctx"] = ctx.numpy()

    def run(controller, tag, steps):
        ref_ptp.register_attention_control(model, controller)
        for s in range(steps):
            for i, pair in enumerate(pairs):
                with torch.no_grad():
                    y1 = pair.attn1(xs[i])
                    y2 = pair.attn2(xs[i], context=ctx)
                out[f"{tag}_s{s}_p{i}_self"] = y1.numpy().copy()
                out[f"{tag}_s{s}_p{i}_cross"] = y2.numpy().copy()

    run(None, "dummy", 1)
    ctrl = nt_ns["AttentionReplace"](FWD_PROMPTS, 4, cross_replace_steps={"default_": .5, "lasagna": .25},
                                     self_replace_steps=.5)
    run(ctrl, "replace", 4)
    for key, lst in ctrl.attention_store.items():
        for i, t in enumerate(lst):
            out[f"replace_store_{key}_{i}"] = t.numpy()
    out["replace_num_att_layers"] = np.array(ctrl.num_att_layers)
    ctrl = nt_ns["AttentionRefine"](["a cat eating a burger", "a fluffy cat eating a burger",
                                     "a cat eating a burger at night"], 4, .75, (.25, .75))
    run(ctrl, "refine", 3)
    np.savez_compressed(os.path.join(OUT, "forward.npz"), **out)
    with open(os.path.join(OUT, "forward.json"), "w") as f:
        json.dump({"geom": FWD_GEOM, "prompts": FWD_PROMPTS, "heads": 2, "ctx_dim": 24,
                   "refine_prompts": ["a cat eating a burger", "a fluffy cat eating a burger",
                                      "a cat eating a burger at night"]}, f, indent=1)
    print("forward:", len(out), "arrays")


# --------------------------------------------------------------------------- LocalBlend
LB_CASES = [
    # (flavour, prompts, words, kwargs, calls)
    ("main", ["a cat sitting on a car", "a dog sitting on a car"], ("cat", "dog"), {}, 1),
    ("null", ["a cat sitting on a car", "a dog sitting on a car"], ("cat", "dog"), {"start_blend": 0.0}, 1),
    ("null", ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger",
              "a painting of a cat eating a burger", "a painting of a squirrel eating a lasagna"],
     ("squirrel", "lion", "cat", "burger"), {"start_blend": 0.0}, 1),
    ("null", ["a painting of a squirrel eating a burger", "a painting of a lion eating a burger",
              "a painting of a cat eating a burger", "a painting of a squirrel eating a lasagna"],
     (("squirrel",), ("lion",), ("cat",), ("burger", "lasagna")),
     {"start_blend": 0.04, "th": (.3, .5), "substruct_words": ("burger", "burger", "burger", "squirrel")}, 3),
]


def _lb_store(B, prompts, g):
    """attention_store-shaped dict with spatially structured 16x16 cross maps (H=1)."""
    yy, xx = torch.meshgrid(torch.arange(16.), torch.arange(16.), indexing="ij")
    store = {"down_cross": [], "up_cross": [], "mid_cross": []}
    for key, n in (("down_cross", 4), ("up_cross", 3)):
        for _ in range(n):
            logits = torch.randn(B, 16, 16, 77, generator=g)
            for b in range(B):
                for w in range(1, 12):
                    cy, cx = torch.randint(0, 16, (2,), generator=g).tolist()
                    blob = torch.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / 8.0)
                    logits[b, :, :, w] += 4.0 * blob
            maps = logits.reshape(B, 256, 77).softmax(-1) * 3.0  # running sum of 3 steps
            store[key].append(_fp16_exact(maps))
    return store


def gen_localblend():
    out = {}
    cases = []
    g = torch.Generator().manual_seed(4321)
    for ci, (flav, prompts, words, kw, calls) in enumerate(LB_CASES):
        B = len(prompts)
        x_t = torch.randn(B, 4, 64, 64, generator=g)
        store = _lb_store(B, prompts, g)
        ns = load_script_classes("main.py" if flav == "main" else "null_text.py", TOK,
                                 extra_globals={"x_t": x_t})
        lb = ns["LocalBlend"](prompts, words, **kw)
        cur = x_t
        for c in range(calls):
            cur = lb(cur, store)
            out[f"case{ci}_out{c}"] = cur.numpy().copy()
        out[f"case{ci}_x_t"] = x_t.numpy()
        for key in ("down_cross", "up_cross"):
            for i, t in enumerate(store[key]):
                out[f"case{ci}_{key}_{i}"] = t.half().numpy()
        out[f"case{ci}_alpha_layers"] = lb.alpha_layers.reshape(B, 77).numpy()
        if getattr(lb, "substruct_layers", None) is not None:
            out[f"case{ci}_substruct_layers"] = lb.substruct_layers.reshape(B, 77).numpy()
        cases.append({"flavour": flav, "prompts": prompts, "words": words, "kwargs": kw,
                      "calls": calls})
    np.savez_compressed(os.path.join(OUT, "localblend.npz"), **out)
    with open(os.path.join(OUT, "localblend.json"), "w") as f:
        json.dump(cases, f, indent=1)
    print("localblend:", len(out), "arrays")


# --------------------------------------------------------------------------- DDIM
def gen_ddim():
    nt_ns = load_script_classes("null_text.py", TOK,
                                extra_globals={"x_t": torch.zeros(1, 4, 64, 64)})
    betas = torch.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000, dtype=torch.float32) ** 2
    alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)

    class _Cfg:
        num_train_timesteps = 1000

    class _Sched:
        config = _Cfg()
        num_inference_steps = 50

    sched = _Sched()
    sched.alphas_cumprod = alphas_cumprod
    sched.final_alpha_cumprod = alphas_cumprod[0]

    class _Self:
        scheduler = sched

    inv = _Self()
    g = torch.Generator().manual_seed(5)
    out = {"alphas_cumprod": alphas_cumprod.numpy()}
    for t in (980, 500, 20, 0):
        x = torch.randn(2, 4, 8, 8, generator=g)
        eps = torch.randn(2, 4, 8, 8, generator=g)
        out[f"t{t}_x"] = x.numpy()
        out[f"t{t}_eps"] = eps.numpy()
        out[f"t{t}_prev"] = nt_ns["NullInversion"].prev_step(inv, eps, t, x).numpy()
        out[f"t{t}_next"] = nt_ns["NullInversion"].next_step(inv, eps, t, x).numpy()
    np.savez_compressed(os.path.join(OUT, "ddim.npz"), **out)
    print("ddim:", len(out), "arrays")


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(4)
    which = sys.argv[1:] or ["tables", "controllers", "forward", "localblend", "ddim"]
    for w in which:
        globals()[f"gen_{w}"]()
