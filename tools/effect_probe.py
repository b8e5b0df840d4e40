"""Edit-effect probe (GPU): how well the end-to-end checks separate a correct edit from a broken
one.  For configs[1] (Replace + LocalBlend) and configs[2] (Refine + Reweight) it runs the oracle
edit, the oracle no-edit base, the product edit and product NEGATIVE controls (no edit, a wrong
mapper, one edit component switched off), and prints per edit prompt the absolute latent cosine
vs the oracle and the edit-effect cosine cos(x - base, oracle - base) (tests/oracle_runs.py).

    python -u tools/effect_probe.py [steps] [dtype:gain ...]      (e.g. 50 f32:1 f32:4 bf16:1)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "prompt-to-prompt_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import torch  # noqa: E402

from oracle import control as oc  # noqa: E402
from oracle_runs import (base_group, cosine, edit_effect, oracle_controller, oracle_group,  # noqa: E402
                         shifted_replace_mapper)
from p2p_amd import config, controllers  # noqa: E402
from p2p_amd import pipeline as pl  # noqa: E402
from p2p_amd.tokenizer import StandInTokenizer  # noqa: E402


def report(name, got, want, base, pbase=None):
    c = cosine(got, want)
    e = edit_effect(got, want, base)
    line = f"  {name:16s} abs cos {[round(x, 6) for x in c.tolist()]}  effect cos {[round(x, 4) for x in e.tolist()]}"
    if pbase is not None:   # the product's own no-edit run as the product side's base
        pe = cosine(got[1:] - pbase[1:], want[1:] - base[1:])
        line += f"  paired {[round(x, 4) for x in pe.tolist()]}"
    print(line, flush=True)


def sharpen(model, gain):
    """Scale every attention's to_q by gain: logits x gain, peaky maps (test-only model knob)."""
    if gain != 1.0:
        for m in model.unet.modules():
            if type(m).__name__ == "CrossAttention":
                m.to_q.weight.mul_(gain)


def configs1(dev, tok, steps, dtype, gain=1.0):
    model = pl.SyntheticStableDiffusion(device=dev, dtype=dtype)
    sharpen(model, gain)
    prompts = pl.north_star_prompts()
    x_T = pl.seed_latent(0)
    t0 = time.time()
    lb = oc.OracleLocalBlend("null", prompts, pl.BLEND_WORDS, tok)
    lb.alpha = lb.alpha.to(dev)
    want = oracle_group(model, prompts, x_T, oracle_controller("replace", prompts, tok, steps, dev, local_blend=lb),
                        steps)
    t1 = time.time()
    base = base_group(model, prompts, x_T, steps)
    t2 = time.time()
    print(f"configs[1] {dtype} U-Net gain {gain}, {steps} steps: oracle edit {t1 - t0:.1f} s, oracle base {t2 - t1:.1f} s; "
          f"|want - base| / |want| per prompt {[round(x, 4) for x in ((want - base).flatten(1).norm(dim=1) / want.flatten(1).norm(dim=1)).tolist()]}",
          flush=True)

    def run(ctrl):
        t = time.time()
        with config.compute_mode("bf16"):
            out = pl.run_edit_group(model, prompts, ctrl, x_T, num_steps=steps)
        torch.cuda.synchronize()
        return out, time.time() - t

    pbase, _ = run(controllers.EmptyControl())
    variants = {
        "edit": lambda: pl.make_replace_controller(prompts, steps, device=dev),
        "no_edit": lambda: controllers.EmptyControl(),
        "store_only": lambda: controllers.AttentionStore(),
        "wrong_mapper": None,
        "no_self": lambda: pl.make_replace_controller(prompts, steps, self_replace_steps=0.0, device=dev),
        "no_cross": lambda: pl.make_replace_controller(prompts, steps, cross_replace_steps=0.0, device=dev),
        "no_blend": lambda: pl.make_replace_controller(prompts, steps, blend_words=None, device=dev),
    }
    for name, mk in variants.items():
        if name == "wrong_mapper":
            ctrl = pl.make_replace_controller(prompts, steps, device=dev)
            ctrl.mapper = shifted_replace_mapper(ctrl.mapper)
        else:
            ctrl = mk()
        got, dt = run(ctrl)
        report(f"{name} {dt:.1f}s", got, want, base, pbase)


def configs2(dev, tok, steps, dtype, gain=1.0):
    model = pl.SyntheticStableDiffusion(device=dev, dtype=dtype)
    sharpen(model, gain)
    prompts = [pl.REFINE_SOURCE] + pl.REFINE_EDITS
    x_T = pl.seed_latent(20)
    t0 = time.time()
    want = oracle_group(model, prompts, x_T, oracle_controller("refine_reweight", prompts, tok, steps, dev), steps)
    base = base_group(model, prompts, x_T, steps)
    print(f"configs[2] {dtype} U-Net, {steps} steps: oracle runs {time.time() - t0:.1f} s; |want - base| / |want| "
          f"{[round(x, 4) for x in ((want - base).flatten(1).norm(dim=1) / want.flatten(1).norm(dim=1)).tolist()]}",
          flush=True)

    def run(ctrl):
        with config.compute_mode("bf16"):
            return pl.run_edit_group(model, prompts, ctrl, x_T, num_steps=steps)

    def wrong_refine():
        c = pl.make_refine_reweight_controller(prompts, steps, device=dev, tokenizer=tok)
        m = c.prev_controller.mapper.clone()
        m[:, 1:] = c.prev_controller.mapper[:, :-1]
        c.prev_controller.mapper = m
        return c

    pbase = run(controllers.EmptyControl())
    variants = {
        "edit": lambda: pl.make_refine_reweight_controller(prompts, steps, device=dev, tokenizer=tok),
        "no_edit": lambda: controllers.EmptyControl(),
        "no_reweight": lambda: pl.make_refine_reweight_controller(prompts, steps, value=1.0, device=dev, tokenizer=tok),
        "wrong_refine": wrong_refine,
    }
    for name, mk in variants.items():
        report(name, run(mk()), want, base, pbase)


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    runs = sys.argv[2:] or ["f32:1", "bf16:1"]
    dev = torch.device("cuda:0")
    tok = StandInTokenizer()
    for r in runs:
        d, g = r.split(":")
        dtype = {"f32": torch.float32, "bf16": torch.bfloat16}[d]
        configs1(dev, tok, steps, dtype, float(g))
        configs2(dev, tok, steps, dtype, float(g))


if __name__ == "__main__":
    main()
