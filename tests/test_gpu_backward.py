"""Attention backward (p2p_attn_fwd_lse + p2p_attn_bwd through attention._AttentionFn) against
torch autograd of the fp32 reference attention (ptp_utils.py:195-206) on the same inputs -- GPU.

The kernels use bf16 MFMA operands with f32 accumulation, so gradients are checked relative to
their own magnitude: max |grad - ref| <= 3e-2 * max |ref| (bf16 keeps 8 significant bits; dK sums
bf16-rounded dS over up to 4096 queries), and
the cosine of every gradient with the reference >= 0.999.
"""
import pytest
import torch

from p2p_amd import attention, config

pytestmark = pytest.mark.gpu

GEOMS = [  # (N, P, K, heads, d)
    (1, 4096, 4096, 2, 40), (2, 1024, 1024, 2, 80), (2, 256, 256, 4, 160), (1, 64, 64, 8, 160),
    (1, 4096, 77, 2, 40), (2, 1024, 77, 2, 80), (2, 256, 77, 4, 160), (2, 130, 50, 2, 64),
]


def ref_attention(q, k, v, heads, scale):
    N, P, C = q.shape
    d = C // heads
    qh = q.reshape(N, P, heads, d).permute(0, 2, 1, 3)
    kh = k.reshape(N, k.shape[1], heads, d).permute(0, 2, 1, 3)
    vh = v.reshape(N, v.shape[1], heads, d).permute(0, 2, 1, 3)
    p = (qh @ kh.transpose(-1, -2) * scale).softmax(-1)
    return (p @ vh).permute(0, 2, 1, 3).reshape(N, P, C)


@pytest.mark.parametrize("geom", GEOMS, ids=lambda g: "x".join(map(str, g)))
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_attention_backward(cuda, geom, dtype):
    N, P, K, H, d = geom
    g = torch.Generator(device=cuda).manual_seed(P + K + d)
    C = H * d
    q = (2.0 * torch.randn(N, P, C, device=cuda, generator=g)).to(dtype).requires_grad_()
    k = torch.randn(N, K, C, device=cuda, generator=g).to(dtype).requires_grad_()
    v = torch.randn(N, K, C, device=cuda, generator=g).to(dtype).requires_grad_()
    dout = torch.randn(N, P, C, device=cuda, generator=g).to(dtype)
    with config.compute_mode("bf16"):
        o = attention.differentiable_attention(q, k, v, H, d ** -0.5)
    o.backward(dout)
    qr, kr, vr = (x.detach().float().requires_grad_() for x in (q, k, v))
    orf = ref_attention(qr, kr, vr, H, d ** -0.5)
    orf.backward(dout.float())
    assert (o.float() - orf).abs().max().item() <= 2 ** -7 * v.float().abs().max().item()
    for name, got, want in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        got = got.float()
        err = (got - want).abs().max().item()
        scale = want.abs().max().item()
        cos = torch.nn.functional.cosine_similarity(got.flatten(), want.flatten(), dim=0).item()
        assert err <= 3e-2 * scale, (name, err, scale)
        assert cos >= 0.999, (name, cos)


def test_patched_forward_is_differentiable(cuda):
    """The hook's plain path (DummyController, null_text.py:610) carries gradients to the context."""
    from p2p_amd import ptp_utils
    from p2p_amd.unet import CrossAttention
    torch.manual_seed(0)
    blk = CrossAttention(320, 768, heads=8, dim_head=40).to(cuda)

    class M(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.down_blocks = torch.nn.ModuleList([blk])

    class Model:
        unet = M()

    ptp_utils.register_attention_control(Model, None)
    x = torch.randn(1, 256, 320, device=cuda)
    ctx = torch.randn(1, 77, 768, device=cuda, requires_grad=True)
    with config.compute_mode("bf16"):
        y = blk(x, context=ctx)
    y.square().mean().backward()
    assert ctx.grad is not None and torch.isfinite(ctx.grad).all() and ctx.grad.abs().max() > 0
