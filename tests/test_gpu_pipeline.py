"""End-to-end parity of a full 50-step edit group (north star: final latents cos >= 0.999,
LocalBlend masks agreeing on >= 99.9 % of pixels) -- GPU.  On random-init weights an edit moves the
latents by ~2 % of their norm, so the absolute cosine is cleared even without any edit; the
edit-EFFECT cosine (tests/oracle_runs.py: product and oracle displacement from the oracle's
no-edit run) carries the discrimination, with negative controls that must fail it.

Product: ptp_utils.text2image_ldm_stable with the fused null_text AttentionReplace +
LocalBlend (bf16 MFMA kernels).  Checker: the same U-Net weights and seed run through the
oracle's eager fp32 attention + reference controller semantics + oracle DDIM, written out
here as a plain loop (ptp_utils.py:65-76, 129-172).  The oracle runs on the GPU with torch
fp32 ops purely as the checker.
"""
import pytest
import torch

from oracle import control as oc
from oracle import forward as ofw
from oracle_runs import EFFECT_BAR, base_group, check_effect, check_negative, shifted_replace_mapper
from p2p_amd import config, controllers
from p2p_amd import pipeline as pl

pytestmark = pytest.mark.gpu


def oracle_group(model, prompts, x_T, tok, steps=50, guidance=7.5):
    lb = oc.OracleLocalBlend("null", prompts, pl.BLEND_WORDS, tok)
    ctrl = oc.OracleController("null", "replace", prompts, steps, 0.8, 0.4, tok, local_blend=lb, store_self=False)
    dev = model.device
    ctrl.mapper, ctrl.alpha, lb.alpha = ctrl.mapper.to(dev), ctrl.alpha.to(dev), lb.alpha.to(dev)
    ofw.install(model, ctrl)
    B = len(prompts)
    ids = model.tokenizer(prompts, padding="max_length", max_length=77, return_tensors="pt").input_ids.to(dev)
    uids = model.tokenizer([""] * B, padding="max_length", max_length=77, return_tensors="pt").input_ids.to(dev)
    ctx = torch.cat([model.text_encoder(uids)[0], model.text_encoder(ids)[0]])
    lat = x_T.expand(B, 4, 64, 64).to(dev)
    sched = model.scheduler
    sched.set_timesteps(steps)
    ac = sched.alphas_cumprod.to(dev)
    with torch.no_grad():
        for t in sched.timesteps:
            eps = model.unet(torch.cat([lat] * 2), t, encoder_hidden_states=ctx)["sample"].float()
            eu, ec = eps.chunk(2)
            lat = oc.ddim_prev(ac, ac[0], eu + guidance * (ec - eu), int(t), lat)
            lat = ctrl.step_callback(lat)
    return lat, lb


def cosine(a, b):
    a, b = a.flatten(1).double(), b.flatten(1).double()
    return torch.nn.functional.cosine_similarity(a, b, dim=1)


@pytest.mark.parametrize("seed", [0])
def test_edit_group_final_latents(cuda, tok, seed):
    prompts = pl.north_star_prompts()
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.float32)
    x_T = pl.seed_latent(seed)
    with config.compute_mode("bf16"):
        ctrl = pl.make_replace_controller(prompts, 50, device=cuda)
        got = pl.run_edit_group(model, prompts, ctrl, x_T, num_steps=50)
    want, _ = oracle_group(model, prompts, x_T, tok)
    cos = cosine(got, want)
    print("final-latent cosine per prompt:", [round(c, 6) for c in cos.tolist()])
    assert torch.isfinite(got).all()
    assert cos.min().item() >= 0.999, cos
    # the edit's EFFECT: (product - no-edit oracle) along (oracle - no-edit oracle), per edit
    # prompt -- the absolute cosine above is cleared even by a run without any edit
    base = base_group(model, prompts, x_T, 50)
    check_effect("configs[1] f32 U-Net", got, want, base, EFFECT_BAR)
    # negative controls: the same product run with the edit disabled, and with a wrong mapper
    with config.compute_mode("bf16"):
        neg_none = pl.run_edit_group(model, prompts, controllers.EmptyControl(), x_T, num_steps=50)
        ctrl = pl.make_replace_controller(prompts, 50, device=cuda)
        ctrl.mapper = shifted_replace_mapper(ctrl.mapper)
        neg_map = pl.run_edit_group(model, prompts, ctrl, x_T, num_steps=50)
    check_negative("no edit", neg_none, want, base, EFFECT_BAR)
    check_negative("wrong mapper", neg_map, want, base, EFFECT_BAR)
    assert cosine(neg_none, want).min().item() >= 0.999     # (what the absolute bar alone would miss)


def test_edit_group_check_mode_tight(cuda, tok):
    """exact-f32 kernels: the whole 50-step group tracks the oracle far tighter."""
    prompts = pl.north_star_prompts()
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.float32)
    x_T = pl.seed_latent(3)
    with config.compute_mode("f32"):
        ctrl = pl.make_replace_controller(prompts, 50, device=cuda)
        got = pl.run_edit_group(model, prompts, ctrl, x_T, num_steps=50)
    want, _ = oracle_group(model, prompts, x_T, tok)
    cos = cosine(got, want)
    print("check-mode final-latent cosine:", [round(c, 8) for c in cos.tolist()])
    assert cos.min().item() >= 0.99999, cos


def test_cross_kv_cache_bit_identical(cuda):
    """The cross-attention K / V projections are computed once per edit group (ptp_utils._cross_kv:
    the loop's context is one tensor for all steps, ptp_utils.py:158-168): every cached K / V equals
    a fresh projection of the context bit for bit, the cache really served the later steps, and a
    bf16 edit group with the cache is bit-identical to one that recomputes them at every call
    (after a warm-up group, so both runs meet the same library kernels)."""
    from p2p_amd import ptp_utils as pu
    prompts = pl.north_star_prompts()
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.bfloat16)
    x_T = pl.seed_latent(5)
    steps = 6
    calls, fresh_equal = [], []
    orig = pu._cross_kv

    def counting(module, context, w):
        hit = module.__dict__.get("_p2p_kv")
        calls.append(hit is not None and hit[0]() is context and hit[1] == context._version and hit[2] is w)
        kv, rows = orig(module, context, w)
        if calls[-1]:   # a cached K / V against a fresh projection of the same context
            fresh_equal.append(torch.equal(kv, torch.nn.functional.linear(context, w)))
        return kv, rows

    def group(cache):
        pu.CACHE_CROSS_KV = cache
        with config.compute_mode("bf16"):
            return pl.run_edit_group(model, prompts, pl.make_replace_controller(prompts, steps, device=cuda), x_T,
                                     num_steps=steps)
    # MIOpen's default convolution solvers are not run-to-run reproducible (tools/determinism_probe.py:
    # two identical U-Net calls differ by up to 2e-2; every hot-path kernel and the U-Net's GEMMs are):
    # the bit-identity tests run the U-Net's convolutions on PyTorch's native im2col + GEMM path
    # (reproducible, 39 ms per U-Net call; MIOpen's deterministic solvers take 1.25 s)
    det = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        group(False)                    # warm-up: library kernel selection, workspaces
        off1 = group(False)
        pu._cross_kv = counting
        on = group(True)
        pu._cross_kv = orig
        off2 = group(False)
    finally:
        pu._cross_kv = orig
        pu.CACHE_CROSS_KV = True
        torch.backends.cudnn.enabled = det
    n_cross = 16
    assert len(calls) == steps * n_cross
    # the first U-Net call of the group computes, the other steps hit
    assert calls[:n_cross] == [False] * n_cross and all(calls[n_cross:]), calls
    assert len(fresh_equal) == (steps - 1) * n_cross and all(fresh_equal)
    print(f"cache off vs off: equal {torch.equal(off1, off2)} max |diff| {(off1 - off2).abs().max().item():.3e}; "
          f"cache on vs off: equal {torch.equal(on, off1)} max |diff| {(on - off1).abs().max().item():.3e}")
    assert torch.equal(off1, off2), "the uncached pipeline is not run-to-run reproducible"
    assert torch.equal(on, off1)


def test_edit_group_under_inference_mode(cuda):
    """A controller built and run under torch.inference_mode() (its alpha table and the
    loop's context then have no version counter): the per-step cross plan keys the alpha table by
    its storage, the K / V projection cache stands aside, and the edit group is bit-identical to the
    same group under torch.no_grad() (reproducible convolutions, as in the K / V cache test)."""
    prompts = pl.north_star_prompts()
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.bfloat16)
    x_T = pl.seed_latent(9)
    steps = 4
    det = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        with config.compute_mode("bf16"):
            with torch.no_grad():
                want = pl.run_edit_group(model, prompts, pl.make_replace_controller(prompts, steps, device=cuda), x_T,
                                         num_steps=steps)
            with torch.inference_mode():
                ctrl = pl.make_replace_controller(prompts, steps, device=cuda)
                assert ctrl.cross_replace_alpha.is_inference()
                got = pl.run_edit_group(model, prompts, ctrl, x_T, num_steps=steps)
    finally:
        torch.backends.cudnn.enabled = det
    assert torch.equal(got, want)


def test_graphed_runner_bit_identical(cuda):
    """GraphedEditRunner (the DDIM steps replayed from HIP graphs captured after the first batch of
    each size) against the eager runner, for one group per U-Net call and for a GroupBatch of two:
    after the capture, a batch of new seeds equals the eager runner's, and a replay of the first
    batch's seeds equals that first (eager) batch -- final latents and reduced 16x16 cross maps,
    bit for bit (the captured controllers' running sums, blend sums and LocalBlend plan start fresh
    at every replay).  Then release() and a fresh capture, and a runner that keeps every self map
    too (bench.py --store-self), whose averaged self maps equal an eager group's.  The bench's 50 steps: the self-injection window (20), the cross-replace
    window (40) and LocalBlend from step 11 all change inside the run.  Reproducible convolutions,
    as the K / V cache test."""
    prompts = pl.north_star_prompts()
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.bfloat16)
    steps = 50
    det = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        with config.compute_mode("bf16"):
            eager = pl.sweep_batch_runner(model, prompts, steps, device=cuda)
            graphed = pl.sweep_batch_runner(model, prompts, steps, device=cuda, graphed=True)
            assert isinstance(graphed, pl.GraphedEditRunner)
            for G in (1, 2):
                first = [100 + g for g in range(G)]
                want0 = graphed(first)                # eager on the capture stream, then the capture
                plan = graphed.plans[G]
                assert len(plan["graphs"]) == steps
                assert len(plan["kv"]) == 16          # every cross layer's K / V captured once, in step 0
                seeds = [200 + g for g in range(G)]
                for want, got in ((eager(seeds), graphed(seeds)), (want0, graphed(first))):
                    for w, g_ in zip(want, got):
                        assert w.shape == g_.shape
                        assert torch.equal(w, g_), (G, (w - g_).abs().max().item())
            # release(): the next batch runs eagerly and captures again, with the same results
            graphed.release()
            assert not graphed.plans
            again = graphed([300])
            assert 1 in graphed.plans
            for w, g_ in zip(eager([300]), again):
                assert torch.equal(w, g_)
            # the kept self maps (bench.py --store-self): every 32x32 / 16x16 / 8x8 self map stored too
            eager_s = pl.sweep_batch_runner(model, prompts, steps, device=cuda, store_self_maps=True)
            graphed_s = pl.sweep_batch_runner(model, prompts, steps, device=cuda, store_self_maps=True, graphed=True)
            graphed_s([400])
            ctrl = graphed_s.plans[1]["ctrl"]
            assert ctrl.store_self_maps and len(ctrl.attention_store["up_self"]) == 6
            for w, g_ in zip(eager_s([401]), graphed_s([401])):
                assert torch.equal(w, g_)
            want_self = ctrl.get_average_attention()["down_self"][0].clone()
            eager_ctrl = pl.make_replace_controller(prompts, steps, device=cuda, store_self_maps=True)
            pl.run_edit_group(model, prompts, eager_ctrl, pl.seed_latent(401), num_steps=steps)
            assert torch.equal(eager_ctrl.get_average_attention()["down_self"][0], want_self)
    finally:
        torch.backends.cudnn.enabled = det


def test_graphed_runner_refine_reweight_groups(cuda):
    """configs[2]'s controllers through the graphed loop: two prompt groups per U-Net call, each an
    AttentionReweight (equalizer) chained on an AttentionRefine whose 16/32-res cross maps are all
    kept (pipeline.make_refine_reweight_controller), 50 steps -- the final latents and reduced 16x16
    maps bit-identical to the eager runner (reproducible convolutions, as above)."""
    prompts = [pl.REFINE_SOURCE] + pl.REFINE_EDITS
    tok = controllers.get_tokenizer()
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.bfloat16)
    steps = 50

    def make_ctrl():
        return pl.make_refine_reweight_controller(prompts, steps, device=cuda, tokenizer=tok)
    det = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    try:
        with config.compute_mode("bf16"):
            eager = pl.edit_batch_runner(model, prompts, make_ctrl, steps)
            graphed = pl.edit_batch_runner(model, prompts, make_ctrl, steps, graphed=True)
            graphed([500, 501])                       # eager + capture
            ctrl = graphed.plans[2]["ctrl"]
            assert isinstance(ctrl, controllers.GroupBatch) and len(ctrl.members) == 2
            for w, g_ in zip(eager([502, 503]), graphed([502, 503])):
                assert torch.equal(w, g_), (w - g_).abs().max().item()
    finally:
        torch.backends.cudnn.enabled = det
