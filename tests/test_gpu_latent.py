"""Fused latent update (p2p_latent_step: CFG combine + DDIM step + LocalBlend blend, SURVEY §8f
rank 1) against the unfused eager sequence of ptp_utils.py:72-75 / null_text.py:471-479 /
null_text.py:68-70 on the same inputs -- GPU.

The eager reference is written out with the same torch ops and the same host-computed 0-dim
coefficients (f32 tensors), in the U-Net's output dtype, so the fused kernel must match it bit
for bit (torch.equal).  The DDIM coefficients themselves are checked against the oracle's
ddim_prev / ddim_next on CPU in tests/test_oracle.py.
"""
import pytest
import torch

from oracle import control as oc
from p2p_amd import _hip, controllers
from p2p_amd.ddim import DDIMScheduler

pytestmark = pytest.mark.gpu


def sched():
    s = DDIMScheduler(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear", clip_sample=False,
                      set_alpha_to_one=False)
    s.set_timesteps(50)
    return s


def eager(eps, x, coeffs, guidance, mask):
    dev = x.device
    sb, sa, sp, s1p = (torch.tensor(c, dtype=torch.float32, device=dev) for c in coeffs)
    if guidance is not None:
        eu, ec = eps.chunk(2)
        noise = eu + guidance * (ec - eu)
    else:
        noise = eps
    x0 = (x - sb * noise) / sa
    out = sp * x0 + s1p * noise
    if mask is not None:
        m = mask[:, None].to(out.dtype)
        out = out[:1] + m * (out - out[:1])
        out = torch.cat([out[:1], out[1:]])
    return out


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("B", [2, 4])
@pytest.mark.parametrize("with_mask", [False, True])
@pytest.mark.parametrize("t", [980, 500, 0])
def test_fused_prev_step_bit_exact(cuda, dtype, B, with_mask, t):
    g = torch.Generator(device=cuda).manual_seed(B * 1000 + t)
    eps = torch.randn(2 * B, 4, 64, 64, device=cuda, generator=g).to(dtype)
    x = torch.randn(B, 4, 64, 64, device=cuda, generator=g)
    mask = (torch.rand(B, 64, 64, device=cuda, generator=g) > 0.5).to(torch.uint8) if with_mask else None
    coeffs = sched().prev_coeffs(t)
    got = _hip.latent_step(eps, x, torch.empty_like(x), coeffs, 7.5, mask)
    want = eager(eps, x, coeffs, 7.5, mask)
    assert want.dtype == torch.float32
    assert torch.equal(got, want), (got - want).abs().max().item()


def test_fused_step_in_place_and_no_cfg(cuda):
    g = torch.Generator(device=cuda).manual_seed(7)
    eps = torch.randn(3, 4, 32, 32, device=cuda, generator=g)
    x = torch.randn(3, 4, 32, 32, device=cuda, generator=g)
    coeffs = sched().next_coeffs(500)
    want = eager(eps, x, coeffs, None, None)
    _hip.latent_step(eps, x, x, coeffs, None, None)          # out aliases x
    assert torch.equal(x, want)


def test_fused_step_matches_oracle_ddim(cuda):
    """the coefficient path end to end against the oracle's restatement of null_text.py:471-479."""
    s = sched()
    g = torch.Generator(device=cuda).manual_seed(3)
    eps = torch.randn(4, 4, 64, 64, device=cuda, generator=g)
    x = torch.randn(4, 4, 64, 64, device=cuda, generator=g)
    for t in (980, 20, 0):
        got = _hip.latent_step(eps, x, torch.empty_like(x), s.prev_coeffs(t), None, None)
        want = oc.ddim_prev(s.alphas_cumprod, s.final_alpha_cumprod, eps.cpu(), t, x.cpu())
        assert torch.allclose(got.cpu(), want, rtol=1e-6, atol=1e-6), (t, (got.cpu() - want).abs().max())


def test_mask_only_localblend_matches_full(cuda):
    """p2p_localblend with x_t = NULL writes the same mask the blending call uses."""
    B, H, L = 4, 8, 5
    g = torch.Generator(device=cuda).manual_seed(11)
    maps = [torch.rand(B * H, 256, 77, device=cuda, generator=g) for _ in range(L)]
    alpha = torch.zeros(B, 77, device=cuda)
    alpha[:, 3] = 1
    alpha[1:, 5] = 1
    x = torch.randn(B, 4, 64, 64, device=cuda, generator=g)
    m_full = torch.empty(B, 64, 64, dtype=torch.uint8, device=cuda)
    m_only = torch.empty_like(m_full)
    ws = torch.empty(B * 2 * L * H * 256, device=cuda)
    xb = x.clone()
    _hip.localblend(maps, H, alpha, None, 0.3, 0.3, xb, ws, mask_out=m_full)
    _hip.localblend(maps, H, alpha, None, 0.3, 0.3, None, ws, mask_out=m_only)
    assert torch.equal(m_full, m_only)
    # and the fused step's blend with that mask equals blending after an unblended step
    eps = torch.randn(2 * B, 4, 64, 64, device=cuda, generator=g)
    coeffs = sched().prev_coeffs(500)
    fused = _hip.latent_step(eps, x, torch.empty_like(x), coeffs, 7.5, m_only)
    plain = _hip.latent_step(eps, x, torch.empty_like(x), coeffs, 7.5, None)
    _hip.localblend(maps, H, alpha, None, 0.3, 0.3, plain, ws)
    assert torch.equal(fused, plain)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
@pytest.mark.parametrize("sub", [False, True], ids=["nosub", "substruct"])
@pytest.mark.parametrize("groups", [(True,), (True, False, True)], ids=["one_group", "three_groups"])
def test_latent_step_builds_folded_blend_mask(cuda, dtype, sub, groups):
    """LocalBlend in the latent-update launch (p2p_latent_step with blend sums, one kernel per
    step): bit-identical to building the mask from the same folded word sums with
    p2p_localblend (word_sums_ready) and blending with it in the mask-reading latent step."""
    gs, H, L = 4, 8, 5
    G = len(groups)
    B = G * gs
    g = torch.Generator(device=cuda).manual_seed(17 + G + 2 * sub)
    eps = torch.randn(2 * B, 4, 64, 64, device=cuda, generator=g).to(dtype)
    x = torch.randn(B, 4, 64, 64, device=cuda, generator=g)
    coeffs = sched().prev_coeffs(500)
    maps = [torch.zeros(gs * H, 256, 77, device=cuda) for _ in range(L)]   # not read (word sums ready)
    alpha = torch.ones(gs, 77, device=cuda)
    subt = torch.ones(gs, 77, device=cuda) if sub else None
    blend, masks = [], []
    for gi, on in enumerate(groups):
        # smooth-ish positive word sums, so the pooled maps cross the thresholds in many places
        # (one spatial field per prompt shared by its L*H maps, with per-map noise: the mean over
        # the maps keeps the field's structure)
        base = torch.rand(gs * 2, 1, 4, 4, device=cuda, generator=g) ** 3
        field = torch.nn.functional.interpolate(base, size=(16, 16), mode="bilinear", align_corners=False)
        sums = field.reshape(gs, 2, 1, 256) * (0.8 + 0.4 * torch.rand(gs, 2, L * H, 256, device=cuda, generator=g))
        sums = sums.contiguous()
        if not sub:
            sums[:, 1] = 0
        fm = controllers.FoldedBlendMask(maps, H, alpha, subt, 0.5, 0.45, (64, 64), sums)
        blend.append(fm.latent_entry() if on else None)
        masks.append(fm.materialize() if on else torch.zeros(gs, 64, 64, dtype=torch.uint8, device=cuda))
    got = _hip.latent_step(eps, x, torch.empty_like(x), coeffs, 7.5, None, gs if G > 1 else 0, None, blend)
    gb = torch.tensor([1 if on else 0 for on in groups], dtype=torch.uint8, device=cuda)
    want = _hip.latent_step(eps, x, torch.empty_like(x), coeffs, 7.5, torch.cat(masks), gs if G > 1 else 0,
                            gb if G > 1 else None)
    frac = torch.cat(masks).float().mean().item()
    assert 0.05 < frac < 0.95, frac        # the masks are neither empty nor full
    assert torch.equal(got, want), (got - want).abs().max().item()
    with pytest.raises(_hip.HipError):      # out may not alias x in the fused form
        _hip.latent_step(eps, x, x, coeffs, 7.5, None, gs if G > 1 else 0, None, blend)


def torch_blend_mask(sums, th_pool, th_sub, size, sub):
    """null_text.py:41-67 restated in float64 torch on word sums that are already taken
    (sums [B, 2, L*H, 256]: plane 0 the alpha words, plane 1 the substruct words): mean over the
    L*H maps, 3x3 max-pool (alpha plane only), nearest upsample, max-normalise, threshold, then
    mask[:1] + mask, and substruct: mask * ~(sub[:1] + sub).  Returns the mask and, per pixel, the
    distance of the deciding normalised values from their thresholds."""
    import torch.nn.functional as F

    def plane(i, pool, th):
        m = sums[:, i].double().mean(1).reshape(-1, 1, 16, 16)
        if pool:
            m = F.max_pool2d(m, (3, 3), (1, 1), padding=(1, 1))
        m = F.interpolate(m, size=size)
        m = (m / m.amax(dim=(2, 3), keepdim=True))[:, 0]
        return m.gt(th), (m - th).abs()

    mask, dist = plane(0, True, th_pool)
    mask = mask[:1] | mask
    dist = torch.minimum(dist, dist[:1])
    if sub:
        s, sd = plane(1, False, th_sub)
        mask = mask & ~(s[:1] | s)
        dist = torch.minimum(dist, torch.minimum(sd, sd[:1]))
    return mask, dist


@pytest.mark.parametrize("sub", [False, True], ids=["nosub", "substruct"])
def test_folded_blend_mask_matches_torch_restatement(cuda, sub):
    """The mask builder itself (the wave-per-plane mean and the on-the-fly pooling of
    build_blend_mask, shared by latent_blend_kernel and blend_finalize_kernel) against a float64
    torch restatement of null_text.py:41-67 on the same folded word sums: every pixel equal except
    where a deciding value sits within 1e-5 of its threshold (f32 vs f64 rounding)."""
    gs, H, L = 4, 8, 5
    g = torch.Generator(device=cuda).manual_seed(41 + sub)
    maps = [torch.zeros(gs * H, 256, 77, device=cuda) for _ in range(L)]
    alpha = torch.ones(gs, 77, device=cuda)
    subt = torch.ones(gs, 77, device=cuda) if sub else None
    worst = 0
    for trial in range(4):
        base = torch.rand(gs * 2, 1, 4, 4, device=cuda, generator=g) ** 3
        field = torch.nn.functional.interpolate(base, size=(16, 16), mode="bilinear", align_corners=False)
        sums = field.reshape(gs, 2, 1, 256) * (0.8 + 0.4 * torch.rand(gs, 2, L * H, 256, device=cuda, generator=g))
        sums = sums.contiguous()
        if not sub:
            sums[:, 1] = 0
        for th_pool, th_sub in ((0.3, 0.3), (0.5, 0.45)):
            got = controllers.FoldedBlendMask(maps, H, alpha, subt, th_pool, th_sub, (64, 64), sums).materialize()
            want, dist = torch_blend_mask(sums, th_pool, th_sub, (64, 64), sub)
            diff = (got != 0) != want
            assert 0.05 < want.float().mean().item() < 0.95
            assert bool((dist[diff] < 1e-5).all()), dist[diff]
            worst = max(worst, int(diff.sum()))
    print(f"folded LocalBlend mask vs float64 torch: at most {worst} near-threshold pixels differ")
    assert worst <= 4


@pytest.mark.parametrize("hw", [(63, 63), (64, 62), (12, 12)], ids=["63x63", "64x62", "12x12"])
def test_latent_step_odd_shapes_fall_back_to_mask_path(cuda, hw):
    """Latents the one-launch LocalBlend does not take (H*W not a multiple of 4, or smaller than
    the 16x16 maps) go through p2p_localblend's mask + the mask-reading latent step
    (ptp_utils._fused_latent_step) instead of failing: the result equals that two-launch path."""
    from types import SimpleNamespace
    from p2p_amd import ptp_utils
    gs, H, L = 4, 8, 5
    g = torch.Generator(device=cuda).manual_seed(5)
    maps = [torch.zeros(gs * H, 256, 77, device=cuda) for _ in range(L)]
    alpha = torch.ones(gs, 77, device=cuda)
    sums = (0.5 + torch.rand(gs, 2, L * H, 256, device=cuda, generator=g)).contiguous()
    sums[:, 1] = 0
    eps = torch.randn(2 * gs, 4, *hw, device=cuda, generator=g)
    x = torch.randn(gs, 4, *hw, device=cuda, generator=g)
    s = sched()
    t = int(s.timesteps[10])

    class Ctrl:
        def fused_step_mask(self):
            return True, lambda size: controllers.FoldedBlendMask(maps, H, alpha, None, 0.3, 0.3, size, sums)

    model = SimpleNamespace(scheduler=s)
    eu, ec = eps.chunk(2)
    got = ptp_utils._fused_latent_step(model, Ctrl(), eps, eu, ec, x, t, 7.5)
    mask = controllers.FoldedBlendMask(maps, H, alpha, None, 0.3, 0.3, hw, sums).materialize()
    want = _hip.latent_step(eps, x, torch.empty_like(x), s.prev_coeffs(t), 7.5, mask)
    assert torch.equal(got, want)
