"""Prompt-group batching (controllers.GroupBatch, BASELINE.json configs[2]) -- GPU.

G edit groups denoised in one U-Net batch must give each group what it gets when it runs alone
(the reference's one-group-per-call loop, main.py:425-444): final latents, the AttentionStore
running sums of every stored layer, and the LocalBlend effect.  Exact-f32 check mode so the only
difference left is the batch size seen by the U-Net's own GEMMs/convolutions.
"""
import pytest
import torch

from p2p_amd import config, controllers, null_text
from p2p_amd import pipeline as pl

pytestmark = pytest.mark.gpu

STEPS = 8


def group_specs(tok, dev):
    """(prompts, controller factory, seed) for two different groups: Replace + LocalBlend, and
    Reweight chained on Refine (configs[2])."""
    rep = pl.north_star_prompts()
    ref = [pl.REFINE_SOURCE] + pl.REFINE_EDITS

    def make_replace():
        lb = null_text.LocalBlend(rep, pl.BLEND_WORDS, start_blend=0.5 * STEPS / 50, tokenizer=tok, device=dev)
        c = null_text.AttentionReplace(rep, STEPS, 0.8, 0.4, local_blend=lb, tokenizer=tok, device=dev)
        c.store_self_maps = False
        return c

    def make_refine():
        return pl.make_refine_reweight_controller(ref, STEPS, device=dev, tokenizer=tok)

    return [(rep, make_replace, 11), (ref, make_refine, 12)]


def cosine(a, b):
    return torch.nn.functional.cosine_similarity(a.flatten(1).double(), b.flatten(1).double(), dim=1)


def test_group_batch_matches_single_groups(cuda, tok):
    model = pl.SyntheticStableDiffusion(device=cuda, dtype=torch.float32)
    specs = group_specs(tok, cuda)
    with config.compute_mode("f32"):
        members = [make() for _, make, _ in specs]
        batch = controllers.GroupBatch(members)
        got = pl.run_edit_groups(model, [p for p, _, _ in specs], batch, [pl.seed_latent(s) for _, _, s in specs],
                                 num_steps=STEPS)
        singles, single_ctrls = [], []
        for prompts, make, seed in specs:
            c = make()
            singles.append(pl.run_edit_group(model, prompts, c, pl.seed_latent(seed), num_steps=STEPS))
            single_ctrls.append(c)
    want = torch.cat(singles)
    cos = cosine(got, want)
    print("batched vs single-group final-latent cosine:", [round(x, 8) for x in cos.tolist()])
    assert cos.min().item() >= 0.99999, cos
    # every member's store == its single-group run's store
    for m, s in zip(members, single_ctrls):
        assert m.cur_step == s.cur_step == STEPS
        am, as_ = m.get_average_attention(), s.get_average_attention()
        for key in as_:
            assert len(am[key]) == len(as_[key]), key
            for x, y in zip(am[key], as_[key]):
                assert torch.allclose(x, y, rtol=1e-3, atol=1e-5), (key, (x - y).abs().max().item())
    # LocalBlend acted in group 0 (the edit latents' blended region equals the source's)
    assert members[0].local_blend.counter == STEPS


def test_group_batch_rejects_materialised_members(cuda, tok):
    class Custom(controllers.AttentionStore):
        def forward(self, attn, is_cross, place_in_unet):
            return attn
    with pytest.raises(ValueError):
        controllers.GroupBatch([Custom()], group_size=4)
