"""Full-size (BASELINE.json configs[1] shapes: SD-v1.4 512x512, bf16 U-Net, batch 8) properties of
the product path that hold independently of the oracle -- GPU.

AttentionStore keeps every self and cross map with P <= 32^2 (main.py:129-142, self maps on as in
the reference default).  Per step each stored probability row sums to 1, so after s steps the
running sum's rows sum to s and get_average_attention's rows to 1 (main.py:144-149) -- for every
self map (null_text's self injection copies the source's rows, still normalised) and for the
source prompt's cross maps (the edits rewrite only the edit prompts' rows, main.py:187-193).
The maps are non-negative, the LocalBlend mask is binary, the latents finite."""
import pytest
import torch

from p2p_amd import pipeline as pl

pytestmark = pytest.mark.gpu

STEPS = 3


@pytest.fixture(scope="module")
def model():
    return pl.SyntheticStableDiffusion(device=torch.device("cuda"), dtype=torch.bfloat16)


def test_running_sums_are_normalised_at_full_size(model):
    prompts = pl.north_star_prompts()
    ctrl = pl.make_replace_controller(prompts, STEPS, store_self_maps=True, device=torch.device("cuda"))
    with torch.no_grad():
        lat = pl.run_edit_group(model, prompts, ctrl, pl.seed_latent(3), num_steps=STEPS)
    torch.cuda.synchronize()
    assert torch.isfinite(lat).all()
    B, H = len(prompts), 8
    store = ctrl.attention_store
    seen = {"self": 0, "cross": 0}
    for key, maps in store.items():
        kind = key.split("_")[1]
        for m in maps:
            assert m.shape[0] == B * H and m.shape[1] <= 32 ** 2
            assert m.min().item() >= 0.0
            rows = m.sum(-1)                              # [B*H, P]: running sum over STEPS steps
            check = rows if kind == "self" else rows[:H]  # cross: the source prompt's rows
            err = (check - STEPS).abs().max().item()
            assert err < 2e-3 * STEPS, (key, tuple(m.shape), err)
            seen[kind] += 1
    # stored layers per kind (P <= 32^2): down 4 (G2, G2, G3, G3), mid 1 (G4), up 6 (G5 x3, G6 x3)
    assert seen == {"self": 11, "cross": 11}, seen
    avg = ctrl.get_average_attention()
    for key, maps in avg.items():
        for m in maps:
            rows = m.sum(-1) if key.endswith("self") else m.sum(-1)[:H]
            assert (rows - 1).abs().max().item() < 2e-3, key


def test_localblend_mask_is_binary_at_full_size(model):
    """null_text.py:53-70 on the full-size running sums: the mask (source OR own, thresholded
    after the max-normalisation) is binary and marks the source's blend word region in every
    prompt (mask[:1] + mask)."""
    from p2p_amd import controllers as c
    prompts = pl.north_star_prompts()
    ctrl = pl.make_replace_controller(prompts, STEPS, device=torch.device("cuda"))
    with torch.no_grad():
        pl.run_edit_group(model, prompts, ctrl, pl.seed_latent(4), num_steps=STEPS)
    lb = ctrl.local_blend
    mask = c.fused_blend_mask(ctrl.attention_store, lb._alpha_flat, None, lb.th[0], lb.th[1], (64, 64))
    torch.cuda.synchronize()
    assert mask.shape == (len(prompts), 64, 64)
    vals = set(torch.unique(mask).tolist())
    assert vals <= {0, 1}, vals
    assert mask.sum().item() > 0
    # every prompt's mask contains the source prompt's
    assert ((mask[:1] == 1) <= (mask == 1)).all()
