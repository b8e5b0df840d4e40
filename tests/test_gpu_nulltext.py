"""Null-text inversion (BASELINE.json configs[4]; null_text.py:469-628) on the HIP attention
forward + backward, against the oracle's restatement with torch autograd through the eager fp32
patched attention on the same U-Net weights -- GPU.

Short schedule (4 DDIM steps, 3 Adam steps each) at 512x512 (64x64 latent): the product's
gradients come from bf16 MFMA kernels, so the optimisation trajectories agree to a cosine, not
bit for bit.  Then the P2P edit with the per-step null embeddings (the notebook's call of
text2image_ldm_stable with uncond_embeddings) runs on the fused kernels.
"""
import pytest
import torch

from oracle import forward as ofw
from oracle import nulltext as ont
from p2p_amd import config, null_text
from p2p_amd import pipeline as pl
from p2p_amd import ptp_utils

pytestmark = pytest.mark.gpu

STEPS, INNER = 4, 3
PROMPT = "a painting of a squirrel eating a burger"


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item()


@pytest.mark.parametrize("use_graphs", [True, False], ids=["graphed", "eager"])
def test_null_text_inversion_matches_oracle(cuda, use_graphs):
    """graphed: every inner Adam step replayed from one captured HIP graph (the default);
    eager: the reference's loop as written."""
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.float32)
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(1, 4, 64, 64, generator=g).to(cuda)
    with config.compute_mode("bf16"):
        inv = null_text.NullInversion(model, num_ddim_steps=STEPS, use_graphs=use_graphs)
        (_, rec), x_T, embs = inv.invert(x0, PROMPT, num_inner_steps=INNER, early_stop_epsilon=1e-5)
        prod_traj = inv.ddim_loop(x0)
    assert rec is None and len(embs) == STEPS and all(e.shape == (1, 77, 768) for e in embs)

    # oracle: same weights, eager fp32 attention, autograd
    ofw.install(model, None)
    sched = model.scheduler
    sched.set_timesteps(STEPS)
    uncond, cond = inv.context.chunk(2)
    traj = ont.ddim_loop(model.unet, sched.alphas_cumprod.to(cuda), sched.final_alpha_cumprod.to(cuda),
                         sched.timesteps, cond, x0, STEPS)
    want_embs, _ = ont.null_optimization(model.unet, sched.alphas_cumprod.to(cuda), sched.final_alpha_cumprod.to(cuda),
                                         sched.timesteps, uncond, cond, traj, STEPS, INNER, 1e-5)
    for a, b in zip(prod_traj, traj):
        assert cos(a, b) >= 0.9999
    assert cos(x_T, traj[-1]) >= 0.9999
    # (with 4 steps the last timestep is 0, where alpha_prev == alpha_t (final_alpha_cumprod =
    # alphas_cumprod[0]) so x_prev == x_t, the loss has no gradient and the last embedding equals
    # the previous one -- in the reference as here)
    u0 = uncond[:1]
    for i, (e, w) in enumerate(zip(embs, want_embs)):
        d_prod, d_want = e - u0, w - u0                  # what the optimiser moved
        print(f"step {i}: |update| {d_want.norm().item():.4f}, cos(updates) {cos(d_prod, d_want):.5f}, "
              f"cos(embeddings) {cos(e, w):.7f}")
        assert cos(e, w) >= 0.9999
        assert cos(d_prod, d_want) >= 0.998     # measured >= 0.99946 (profiles/r02b, r03)


def test_null_text_inversion_full_schedule(cuda):
    """configs[4] at its stated schedule: 50 DDIM steps x 10 Adam steps (null_text.py:591-618,
    early stop 1e-5), graphed product path vs the oracle's fp32 autograd on the same weights.  Over
    50 dependent steps the bf16-kernel gradients drift a little: the per-step bars are cosine >= 0.999
    on the optimiser's updates and >= 0.9995 on the embeddings themselves (measured 0.9995 and 0.99967,
    profiles/r02b/nulltext_full_schedule.log); the DDIM trajectory is a forward-only quantity and
    stays at >= 0.9999."""
    steps, inner = 50, 10
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.float32)
    g = torch.Generator().manual_seed(7)
    x0 = torch.randn(1, 4, 64, 64, generator=g).to(cuda)
    with config.compute_mode("bf16"):
        inv = null_text.NullInversion(model, num_ddim_steps=steps, use_graphs=True)
        (_, _), x_T, embs = inv.invert(x0, PROMPT, num_inner_steps=inner, early_stop_epsilon=1e-5)
        prod_traj = inv.ddim_loop(x0)
    ofw.install(model, None)
    sched = model.scheduler
    sched.set_timesteps(steps)
    uncond, cond = inv.context.chunk(2)
    ac, fa = sched.alphas_cumprod.to(cuda), sched.final_alpha_cumprod.to(cuda)
    traj = ont.ddim_loop(model.unet, ac, fa, sched.timesteps, cond, x0, steps)
    want_embs, _ = ont.null_optimization(model.unet, ac, fa, sched.timesteps, uncond, cond, traj, steps, inner, 1e-5)
    assert min(cos(a, b) for a, b in zip(prod_traj, traj)) >= 0.9999
    u0 = uncond[:1]
    worst_e, worst_u = 1.0, 1.0
    for i, (e, w) in enumerate(zip(embs, want_embs)):
        worst_e = min(worst_e, cos(e, w))
        if (w - u0).norm().item() > 1e-6:
            worst_u = min(worst_u, cos(e - u0, w - u0))
    print(f"50x10 null-text: worst cos(embeddings) {worst_e:.6f}, worst cos(updates) {worst_u:.4f}")
    assert worst_e >= 0.9995
    assert worst_u >= 0.999


@pytest.mark.parametrize("steps,inner", [(4, 2), (50, 10)], ids=["4x2", "50x10"])
def test_edit_with_null_embeddings(cuda, tok, steps, inner):
    """configs[4]'s second half: the P2P edit after inversion -- per-step null embeddings (the
    notebook's text2image_ldm_stable(..., uncond_embeddings=...) call; ptp_utils.py:129-172 plus
    the context swap of null_text.py:574-618's caller) + fused AttentionReplace + null_text
    LocalBlend, against the ORACLE run with the SAME null embeddings, latent and weights (eager fp32
    attention, reference controller semantics, oracle DDIM / LocalBlend).  50x10 is configs[4]'s
    stated schedule (50 DDIM steps, 10 Adam steps per step, then the 50-step edit).  Bars: final
    latents cosine >= 0.999 per prompt (north star) and the edit-effect cosine against the
    oracle's no-edit run with the same embeddings >= 0.99; the same run without the edit must
    fail it."""
    from oracle import control as oc
    from oracle_runs import EFFECT_BAR, base_group, check_effect, check_negative, cosine, oracle_controller, \
        oracle_group
    from p2p_amd import controllers
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.float32)
    g = torch.Generator().manual_seed(6)
    x0 = torch.randn(1, 4, 64, 64, generator=g).to(cuda)
    prompts = [PROMPT, "a painting of a lion eating a burger"]
    with config.compute_mode("bf16"):
        inv = null_text.NullInversion(model, num_ddim_steps=steps)
        _, x_T, embs = inv.invert(x0, PROMPT, num_inner_steps=inner)
        lb = null_text.LocalBlend(prompts, ("squirrel", "lion"), start_blend=0.2, tokenizer=tok, device=cuda)
        ctrl = null_text.AttentionReplace(prompts, steps, 0.8, 0.4, local_blend=lb, tokenizer=tok, device=cuda)
        lat, _ = ptp_utils.text2image_ldm_stable(model, prompts, ctrl, num_inference_steps=steps, latent=x_T,
                                                 uncond_embeddings=embs)
        neg, _ = ptp_utils.text2image_ldm_stable(model, prompts, controllers.EmptyControl(), num_inference_steps=steps,
                                                 latent=x_T, uncond_embeddings=embs)
    assert lat.shape == (2, 4, 64, 64) and torch.isfinite(lat).all()
    assert ctrl.cur_step == steps
    # the oracle, same null embeddings (the product's), same x_T
    olb = oc.OracleLocalBlend("null", prompts, ("squirrel", "lion"), tok, start_blend=0.2)
    olb.alpha = olb.alpha.to(cuda)
    octrl = oracle_controller("replace", prompts, tok, steps, cuda, local_blend=olb)
    ue = [e.detach() for e in embs]
    want = oracle_group(model, prompts, x_T, octrl, steps, uncond_embeddings=ue)
    c = cosine(lat, want)
    print(f"edit after null-text ({steps}x{inner}): final-latent cosine vs oracle {[round(x, 6) for x in c.tolist()]}")
    assert c.min().item() >= 0.999
    base = base_group(model, prompts, x_T, steps, uncond_embeddings=ue)
    check_effect(f"edit after null-text ({steps}x{inner})", lat, want, base, EFFECT_BAR)
    check_negative("no edit", neg, want, base, EFFECT_BAR)
