"""Attention entry points used by the patched ``CrossAttention.forward``.

* ``plain_attention``        -- no controller work (``DummyController``, uncond passes);
* ``materialized_attention`` -- the reference protocol for controllers that edit a
  materialised probability tensor (``controller(attn, is_cross, place)``,
  ptp_utils.py:204-206): probabilities and P.V both run as HIP kernels, the controller
  sees an f32 ``[N*H, P, K]`` tensor exactly like the reference's.

Fused controllers (this package's AttentionStore / AttentionControlEdit family) bypass
both and launch one edit-aware kernel per call (controllers.py).
"""
from __future__ import annotations

import torch

from . import _hip
from . import config


class _AttentionFn(torch.autograd.Function):
    """softmax(Q K^T * scale) V with its gradient on the HIP kernels (p2p_attn_fwd_lse /
    p2p_attn_bwd) -- what null-text inversion back-propagates through (null_text.py:587-598)."""

    @staticmethod
    def forward(ctx, q, k, v, heads, scale):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        N, P, _ = q.shape
        o = torch.empty_like(q)
        lse = torch.empty(N * heads, P, dtype=torch.float32, device=q.device)
        _hip.attn_fwd_lse(q, k, v, o, heads, scale, lse)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.heads, ctx.scale = heads, scale
        return o

    @staticmethod
    def backward(ctx, dout):
        q, k, v, o, lse = ctx.saved_tensors
        dout = dout.contiguous().to(q.dtype)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)                 # written by the kernels (f32 accumulation inside)
        dv = torch.empty_like(v)
        delta = torch.empty_like(lse)
        _hip.attn_bwd(q, k, v, o, dout, lse, ctx.heads, ctx.scale, dq, dk, dv, delta)
        return dq, dk, dv, None, None


def differentiable_attention(q, k, v, heads, scale):
    if config.COMPUTE != "bf16":
        raise NotImplementedError("the attention backward runs on the bf16 kernels only (compute='bf16')")
    return _AttentionFn.apply(q, k, v, heads, scale)


def plain_attention(q, k, v, heads, scale, out=None):
    if torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad):
        return differentiable_attention(q, k, v, heads, scale)
    out = torch.empty_like(q) if out is None else out
    if k.shape[1] <= _hip.MAX_KEYS_CROSS:
        # one prompt group without an edit program: every entry uses its own probabilities
        _hip.cross_attn(q, k, v, out, heads, scale, [(0, q.shape[0], None, None)], compute=config.COMPUTE)
    else:
        _hip.self_attn(q, k, v, out, heads, scale, compute=config.COMPUTE)
    return out


def attention_probs(q, k, heads, scale, mask=None):
    """softmax(Q K^T * scale) as [N*H, P, K] f32 (ptp_utils.py:195-204)."""
    N, P, _ = q.shape
    K = k.shape[1]
    probs = torch.empty(N * heads, P, K, dtype=torch.float32, device=q.device)
    key_mask = None
    if mask is not None:
        key_mask = mask.reshape(N, -1).to(device=q.device, dtype=torch.uint8).contiguous()
        if key_mask.shape[1] != K:
            raise ValueError(f"mask has {key_mask.shape[1]} keys, attention has {K}")
    _hip.attn_probs(q, k, heads, scale, probs, compute=config.COMPUTE, key_mask=key_mask)
    return probs


def attention_pv(probs, v, heads, n_query, out_dtype):
    N = v.shape[0]
    out = torch.empty(N, n_query, v.shape[2], dtype=out_dtype, device=v.device)
    _hip.attn_pv(probs.contiguous(), v, out, heads, compute=config.COMPUTE)
    return out


def materialized_attention(controller, q, k, v, heads, scale, is_cross, place_in_unet, mask=None):
    probs = attention_probs(q, k, heads, scale, mask)
    probs = controller(probs, is_cross, place_in_unet)
    if probs.dtype != torch.float32:
        probs = probs.float()
    return attention_pv(probs, v, heads, q.shape[1], q.dtype)
