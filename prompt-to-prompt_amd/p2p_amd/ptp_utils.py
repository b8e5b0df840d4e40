"""Drop-in for the reference ``ptp_utils.py``: the attention hook, the sampling loop and the
word/time tables.

``register_attention_control(model, controller)`` keeps the reference's patching rule
(every module whose class is named ``CrossAttention`` under ``unet.{down,mid,up}*``,
ptp_utils.py:223-240) and its forward signature (``:183``), and sets
``controller.num_att_layers`` (``:242``).  The replacement forward keeps the projections as
they are and hands ``q, k, v`` to the controller's fused kernel (controllers.py) -- or, for a
reference-style controller, to the materialised protocol (attention.py).
"""
from __future__ import annotations

import os
from typing import List, Optional

import numpy as np
import torch

from .attention import materialized_attention, plain_attention
from .ptp_words import get_time_words_attention_alpha, get_word_inds, update_alpha_time_word  # noqa: F401


# ------------------------------------------------------------------ sampling loop
def diffusion_step(model, controller, latents, context, t, guidance_scale, low_resource=False, t_unet=None):
    """One CFG denoising step (ptp_utils.py:65-76).  With this library's DDIM scheduler and a
    controller whose step_callback is its own, the CFG combine, the DDIM step and LocalBlend's
    latent blend run as one HIP kernel (p2p_latent_step) -- same result, bit for bit.
    ``t_unet``: the same timestep as a device tensor for the U-Net (a captured step must not copy
    a host timestep to the device); the scheduler keeps reading the host ``t``."""
    tu = t if t_unet is None else t_unet
    if low_resource:
        eps_u = model.unet(latents, tu, encoder_hidden_states=context[0])["sample"]
        eps_c = model.unet(latents, tu, encoder_hidden_states=context[1])["sample"]
        eps = None
    else:
        eps = model.unet(torch.cat([latents] * 2), tu, encoder_hidden_states=context)["sample"]
        eps_u, eps_c = eps.chunk(2)
    fused = _fused_latent_step(model, controller, eps, eps_u, eps_c, latents, t, guidance_scale)
    if fused is not None:
        return fused
    noise_pred = eps_u + guidance_scale * (eps_c - eps_u)
    latents = model.scheduler.step(noise_pred, t, latents)["prev_sample"]
    return controller.step_callback(latents)


def _fused_latent_step(model, controller, eps, eps_u, eps_c, latents, t, guidance_scale):
    from . import _hip
    from .ddim import DDIMScheduler
    if not (isinstance(model.scheduler, DDIMScheduler) and latents.is_cuda and latents.dtype == torch.float32
            and eps_u.dtype in (torch.float32, torch.bfloat16) and hasattr(controller, "fused_step_mask")):
        return None
    ok, mask_fn = controller.fused_step_mask()
    if not ok:
        return None
    if eps is None or not eps.is_contiguous():
        eps = torch.cat([eps_u, eps_c]).contiguous()
    from .controllers import FoldedBlendMask, group_mask_tensor
    x = latents.contiguous()
    out = torch.empty_like(x)
    mask = mask_fn(tuple(x.shape[2:])) if mask_fn is not None else None
    group_size, group_blend, blend = 0, None, None
    folded = mask if isinstance(mask, FoldedBlendMask) else (
        next((m for m in mask[0] if m is not None), None) if isinstance(mask, tuple) and len(mask) == 2 else None)
    if folded is not None and not _blend_launch_ok(x, out, eps, folded):
        # shapes the one-launch LocalBlend does not take: the mask is built by p2p_localblend and
        # the latent step reads it (the same mask, two launches)
        mask = folded.materialize() if isinstance(mask, FoldedBlendMask) else group_mask_tensor(
            mask[0], mask[1], tuple(x.shape[2:]))
    if isinstance(mask, FoldedBlendMask):  # LocalBlend built inside the latent-step launch
        mask, blend = None, [mask.latent_entry()]
    elif isinstance(mask, tuple) and len(mask) == 2:   # prompt-group batch, every blending group folded
        blend = [m.latent_entry() if m is not None else None for m in mask[0]]
        mask, group_size = None, mask[1]
    elif isinstance(mask, tuple):          # prompt-group batch: (mask, group size, groups that blend)
        mask, group_size, group_blend = mask
    return _hip.latent_step(eps, x, out, model.scheduler.prev_coeffs(t), guidance_scale, mask,
                            group_size, group_blend, blend)


def _blend_launch_ok(x, out, eps, folded) -> bool:
    """The one-launch LocalBlend's preconditions (p2p_blend.hip run_latent_step, include/p2p_hip.h):
    whole 4-pixel vectors (H*W % 4 == 0), 16-byte aligned x / out / eps, and a latent at least as
    large as the map resolution (the 3x3-pooled map is nearest-upsampled onto it)."""
    H, W = x.shape[2], x.shape[3]
    res = int(round(folded.sums.shape[-1] ** 0.5))
    return ((H * W) % 4 == 0 and res <= H and res <= W and res * res <= 256
            and (x.data_ptr() | out.data_ptr() | eps.data_ptr()) % 16 == 0)


def latent2image(vae, latents):
    """ptp_utils.py:79-85 (needs a VAE; the synthetic pipeline has none)."""
    latents = 1 / 0.18215 * latents
    image = vae.decode(latents)["sample"]
    image = (image / 2 + 0.5).clamp(0, 1)
    image = image.cpu().permute(0, 2, 3, 1).numpy()
    return (image * 255).astype(np.uint8)


def init_latent(latent, model, height, width, generator, batch_size):
    """ptp_utils.py:88-95: one x_T shared by every prompt of the group."""
    if latent is None:
        latent = torch.randn((1, model.unet.in_channels, height // 8, width // 8), generator=generator)
    latents = latent.expand(batch_size, model.unet.in_channels, height // 8, width // 8).to(model.device)
    return latent, latents


def _encode(model, prompts, encoder):
    ids = model.tokenizer(prompts, padding="max_length", max_length=model.tokenizer.model_max_length,
                          truncation=True, return_tensors="pt").input_ids
    return encoder(ids.to(model.device))[0]


def unet_context(model, context):
    """The context in the U-Net's own dtype, cast once before the sampling loop: a U-Net that
    casts ``encoder_hidden_states`` itself then gets back this same tensor at every step (a cast
    to its own dtype is a no-op), which keeps the cross-attention K / V cache of _cross_kv valid
    across steps."""
    dtype = getattr(model.unet, "dtype", None)
    if not isinstance(dtype, torch.dtype):
        return context
    if isinstance(context, (list, tuple)):
        return type(context)(c.to(dtype) for c in context)
    return context.to(dtype)


@torch.no_grad()
def text2image_ldm(model, prompt: List[str], controller, num_inference_steps: int = 50,
                   guidance_scale: Optional[float] = 7., generator: Optional[torch.Generator] = None,
                   latent: Optional[torch.FloatTensor] = None):
    """ptp_utils.py:98-126 (LDM-256: 32x32 latent, LDMBert context)."""
    register_attention_control(model, controller)
    height = width = 256
    batch_size = len(prompt)
    uncond = _encode(model, [""] * batch_size, model.bert)
    text = _encode(model, prompt, model.bert)
    latent, latents = init_latent(latent, model, height, width, generator, batch_size)
    context = unet_context(model, torch.cat([uncond, text]))
    model.scheduler.set_timesteps(num_inference_steps)
    for t in model.scheduler.timesteps:
        latents = diffusion_step(model, controller, latents, context, t, guidance_scale)
    image = latent2image(model.vqvae, latents) if getattr(model, "vqvae", None) is not None else latents
    return image, latent


@torch.no_grad()
def text2image_ldm_stable(model, prompt: List[str], controller, num_inference_steps: int = 50,
                          guidance_scale: float = 7.5, generator: Optional[torch.Generator] = None,
                          latent: Optional[torch.FloatTensor] = None, low_resource: bool = False,
                          uncond_embeddings=None):
    """ptp_utils.py:129-172.  ``uncond_embeddings`` (per-step list or one tensor) is the
    argument the missing null-text notebook passes for the edit after inversion.  Without a
    VAE on the model the final latents are returned in place of the image."""
    register_attention_control(model, controller)
    height = width = 512
    batch_size = len(prompt)
    text = _encode(model, prompt, model.text_encoder)
    if uncond_embeddings is None:
        uncond = _encode(model, [""] * batch_size, model.text_encoder)
    else:
        uncond = None
    latent, latents = init_latent(latent, model, height, width, generator, batch_size)
    model.scheduler.set_timesteps(num_inference_steps)
    # one context for the whole loop, as ptp_utils.py:158-160 builds it: the cross-attention K / V
    # projections of an unchanged context are then computed once (_project's cache); per-step null
    # embeddings make a new context every step
    context = None if uncond_embeddings is not None else unet_context(
        model, [uncond, text] if low_resource else torch.cat([uncond, text]))
    for i, t in enumerate(model.scheduler.timesteps):
        if uncond_embeddings is not None:
            u = uncond_embeddings[i] if isinstance(uncond_embeddings, (list, tuple)) else uncond_embeddings
            uncond = u.expand(*text.shape)
            context = [uncond, text] if low_resource else torch.cat([uncond, text])
        latents = diffusion_step(model, controller, latents, context, t, guidance_scale, low_resource)
    image = latent2image(model.vae, latents) if getattr(model, "vae", None) is not None else latents
    return image, latent


# ------------------------------------------------------------------ the hook
class DummyController:
    """ptp_utils.py:212-218: identity controller (used by null-text inversion)."""

    def __call__(self, *args):
        return args[0]

    def attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask=None):
        if mask is not None:
            return materialized_attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask)
        return plain_attention(q, k, v, heads, scale)

    def __init__(self):
        self.num_att_layers = 0


FUSE_PROJECTIONS = os.environ.get("P2P_FUSE_QKV", "1") != "0"


def _stacked_weight(module, names):
    """One [sum(out), in] weight for the bias-free projections ``names`` of ``module``
    (diffusers-0.8.1 CrossAttention's to_q/to_k/to_v carry no bias), rebuilt whenever a
    source weight is replaced or modified in place; None when they cannot be stacked."""
    mods = [getattr(module, n, None) for n in names]
    if not all(type(m) is torch.nn.Linear and m.bias is None for m in mods):
        return None
    key = tuple((m.weight.data_ptr(), m.weight._version, m.weight.dtype) for m in mods)
    cache = module.__dict__.setdefault("_p2p_stacked", {})
    hit = cache.get(names)
    if hit is None or hit[0] != key:
        hit = (key, torch.cat([m.weight.detach() for m in mods]))
        cache[names] = hit
    return hit[1]


CACHE_CROSS_KV = os.environ.get("P2P_CACHE_CROSS_KV", "1") != "0"


def _cross_kv(module, context, w):
    """linear(context, [to_k; to_v]) of a cross-attention, computed once per (context, weights):
    the sampling loop hands every U-Net call of an edit group the same context tensor
    (ptp_utils.py:158-168), so its K / V are the same at all 50 steps.  The cache holds the
    context by identity (a weak reference: a new tensor, even at a recycled address, misses) and
    its version counter (an in-place change misses), and the stacked weight object (rebuilt by
    _stacked_weight whenever a projection weight changes).  Not cached: inference-mode tensors (no
    version counter).
    Under stream capture an entry is made and hit only among captures: the first captured call
    records its GEMM in its graph (which recomputes K / V from the static context a replay has
    refilled, e.g. pipeline.GraphedEditRunner's step 0 or null-text's per-step uncond embeddings)
    and the later captured steps read that GEMM's output; an entry made eagerly is never hit by a
    capture (its K / V are of the context's content at that time, not at replay), and a captured
    entry never by an eager call (its K / V exist only once a replay ran).  The SHARED_KV row
    classes need a device read, so captured entries carry none."""
    import weakref
    if not CACHE_CROSS_KV or context.is_inference() or context.requires_grad:
        return torch.nn.functional.linear(context, w), None
    capturing = _capturing(context)
    hit = module.__dict__.get("_p2p_kv")
    if (hit is not None and hit[0]() is context and hit[1] == context._version and hit[2] is w
            and hit[5] == capturing):
        return hit[3], hit[4]
    kv = torch.nn.functional.linear(context, w)
    rows = None if capturing else kv_row_classes(kv)
    module.__dict__["_p2p_kv"] = (weakref.ref(context), context._version, w, kv, rows, capturing)
    return kv, rows


def _capturing(t) -> bool:
    """True while ``t``'s device stream is being captured into a HIP graph."""
    return t.is_cuda and torch.cuda.is_current_stream_capturing()


def kv_row_classes(kv):
    """For each batch row of a cross-attention's K / V projection, the first row of its run of
    bit-identical rows (rows n and n + 1 compared exactly) -- e.g. the uncond prompts "" of a group
    (ptp_utils.py:150-156) give equal context rows, hence equal K and V.  Computed once per cached
    projection (one device -> host read); the controllers turn it into p2p_group's SHARED_KV."""
    flat = kv.reshape(kv.shape[0], -1)
    same = (flat[1:] == flat[:-1]).all(dim=1).tolist()
    rows = [0]
    for i, eq in enumerate(same):
        rows.append(rows[-1] if eq else i + 1)
    return tuple(rows)


def _project(module, x, context, is_cross):
    """q, k, v of ptp_utils.py:186-193.  Outside autograd one GEMM produces them (x read once
    for self-attention, the context once for k and v) and the kernels read q/k/v as strided
    views of its output -- no head split copies (``[b,n,h*d] -> [b*h,n,d]``, :191-193).  A
    cross-attention's k / v of an unchanged context come from the previous call (_cross_kv)."""
    src = context if is_cross else x
    grad = torch.is_grad_enabled() and (x.requires_grad or src.requires_grad)
    if FUSE_PROJECTIONS and not grad and x.is_cuda:
        if is_cross:
            w = _stacked_weight(module, ("to_k", "to_v"))
            if w is not None:
                kv, rows = _cross_kv(module, src, w)
                C = kv.shape[-1] // 2
                k, v = kv[..., :C], kv[..., C:]
                if rows is not None:
                    k._p2p_rows = v._p2p_rows = rows   # (read by the controllers' group hints)
                return module.to_q(x), k, v
        else:
            w = _stacked_weight(module, ("to_q", "to_k", "to_v"))
            if w is not None:
                qkv = torch.nn.functional.linear(x, w)
                C = qkv.shape[-1] // 3
                return qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    return module.to_q(x), module.to_k(src), module.to_v(src)


def _make_forward(module, place_in_unet, controller):
    to_out = module.to_out[0] if type(module.to_out) is torch.nn.modules.container.ModuleList else module.to_out
    attend = getattr(controller, "attention", None)

    def forward(x, context=None, mask=None, encoder_hidden_states=None, attention_mask=None):
        is_cross = context is not None          # only the ``context=`` kwarg counts (:187)
        q, k, v = _project(module, x, context, is_cross)
        if attend is not None:
            out = attend(q, k, v, module.heads, module.scale, is_cross, place_in_unet, mask)
        else:
            out = materialized_attention(controller, q, k, v, module.heads, module.scale, is_cross,
                                         place_in_unet, mask)
        return to_out(out)

    return forward


def register_attention_control(model, controller):
    if controller is None:
        controller = DummyController()

    def walk(net, count, place):
        if net.__class__.__name__ == "CrossAttention":
            net.forward = _make_forward(net, place, controller)
            return count + 1
        if hasattr(net, "children"):
            for child in net.children():
                count = walk(child, count, place)
        return count

    total = 0
    for name, net in model.unet.named_children():
        if "down" in name:
            total += walk(net, 0, "down")
        elif "up" in name:
            total += walk(net, 0, "up")
        elif "mid" in name:
            total += walk(net, 0, "mid")
    controller.num_att_layers = total
