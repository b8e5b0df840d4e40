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
from p2p_amd import _hip
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
