"""The ``null_text.py`` flavour of the controllers (null_text.py:39-401).

Differences from ``main.py`` that the reference carries and this module keeps:
* self-attention injection for maps with up to 32**2 keys (null_text.py:225), and
  ``replace_self_attention`` takes ``place_in_unet``;
* LocalBlend with a ``start_blend`` gate, two thresholds and an optional substruct mask
  (null_text.py:39-102), valid for any number of prompts;
* ``get_equalizer`` with one value per selected word in a single row (null_text.py:340-349);
* ``EmptyControl`` is not an AttentionControl (no counters, null_text.py:105-114).

Three latent bugs of the reference are NOT reproduced: LocalBlend reads
the size from its ``x_t`` argument instead of a global, ``make_controller`` uses its
``blend_words`` argument, and ``SpatialReplace`` counts its own steps.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple, Union

import torch

from . import controllers as _c
from .attention import materialized_attention, plain_attention
from .controllers import aggregate_attention, get_tokenizer, default_device, NotFusable  # noqa: F401
from .ptp_words import get_word_inds

NUM_DDIM_STEPS = 50     # null_text.py:23
GUIDANCE_SCALE = 7.5    # null_text.py:24
MAX_NUM_WORDS = 77      # null_text.py:25


class LocalBlend:
    """null_text.py:39-102."""

    def get_mask(self, maps, alpha, use_pool):
        """Reference-protocol mask of a materialised [B, L*H, 1, 16, 16, W] map stack."""
        import torch.nn.functional as nnf
        k = 1
        maps = (maps * alpha).sum(-1).mean(1)
        if use_pool:
            maps = nnf.max_pool2d(maps, (k * 2 + 1, k * 2 + 1), (1, 1), padding=(k, k))
        mask = nnf.interpolate(maps, size=self._size)
        mask = mask / mask.max(2, keepdims=True)[0].max(3, keepdims=True)[0]
        mask = mask.gt(self.th[1 - int(use_pool)])
        return mask[:1] + mask

    def __call__(self, x_t, attention_store):
        self.counter += 1
        if self.counter > self.start_blend:
            self._size = tuple(x_t.shape[2:])
            sub = self._sub_flat if self.substruct_layers is not None else None
            x_t = _c.fused_local_blend(x_t, attention_store, self._alpha_flat, sub, self.th[0], self.th[1])
        return x_t

    def step_mask(self, attention_store, size, folded=None):
        """What __call__ does to its counter, returning the mask it would blend with (or None
        before start_blend) -- the fused latent-step protocol.  ``folded``: the running word sums
        the cross-attention store epilogue accumulated (AttentionControlEdit._blend_fold)."""
        self.counter += 1
        if self.counter > self.start_blend:
            self._size = tuple(size)
            sub = self._sub_flat if self.substruct_layers is not None else None
            return _c.fused_blend_mask(attention_store, self._alpha_flat, sub, self.th[0], self.th[1], size,
                                       folded)
        return None

    def _fold_tables(self):
        """(alpha [B, W], substruct [B, W] or None) the store epilogue folds the word sums with."""
        return self._alpha_flat, (self._sub_flat if self.substruct_layers is not None else None)

    def __init__(self, prompts: List[str], words, substruct_words=None, start_blend=0.2, th=(.3, .3),
                 tokenizer=None, device=None):
        tokenizer = tokenizer or get_tokenizer()
        device = device or default_device()
        self.alpha_layers = _c._word_alpha_layers(prompts, words, tokenizer).to(device)
        self._alpha_flat = self.alpha_layers.reshape(len(prompts), -1).contiguous()
        if substruct_words is not None:
            self.substruct_layers = _c._word_alpha_layers(prompts, substruct_words, tokenizer).to(device)
            self._sub_flat = self.substruct_layers.reshape(len(prompts), -1).contiguous()
        else:
            self.substruct_layers = None
        self.start_blend = int(start_blend * NUM_DDIM_STEPS)
        self.counter = 0
        self.th = th


LocalBlend._P2P_LIB = True


class EmptyControl:
    """null_text.py:105-114 -- identity, no counters."""

    def step_callback(self, x_t):
        return x_t

    def fused_step_mask(self):
        return (True, None) if _c._owned(self, "step_callback") else (False, None)

    def between_steps(self):
        return

    def __call__(self, attn, is_cross: bool, place_in_unet: str):
        return attn

    def attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask=None):
        if type(self).__call__ is not EmptyControl.__call__ or mask is not None:
            return materialized_attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask)
        return plain_attention(q, k, v, heads, scale)


EmptyControl._P2P_LIB = True


class SpatialReplace(EmptyControl):
    """null_text.py:158-168: copy the source latent into every prompt for the first steps."""

    def step_callback(self, x_t):
        if self.cur_step < self.stop_inject:
            b = x_t.shape[0]
            x_t = x_t[:1].expand(b, *x_t.shape[1:])
        self.cur_step += 1
        return x_t

    def __init__(self, stop_inject: float):
        super().__init__()
        self.stop_inject = int((1 - stop_inject) * NUM_DDIM_STEPS)
        self.cur_step = 0


AttentionControl = _c.AttentionControl
AttentionStore = _c.AttentionStore


class AttentionControlEdit(_c.AttentionControlEdit):
    """null_text.py:217-269."""

    SELF_REPLACE_MAX_KEYS = 32 ** 2

    def replace_self_attention(self, attn_base, att_replace, place_in_unet):
        if att_replace.shape[2] <= self.SELF_REPLACE_MAX_KEYS:
            return attn_base.unsqueeze(0).expand(att_replace.shape[0], *attn_base.shape)
        return att_replace

    def _replace_self(self, attn_base, att_replace, place_in_unet):
        return self.replace_self_attention(attn_base, att_replace, place_in_unet)


AttentionControlEdit._P2P_LIB = True


class AttentionReplace(AttentionControlEdit, _c.AttentionReplace):
    """null_text.py:272-287."""


class AttentionRefine(AttentionControlEdit, _c.AttentionRefine):
    """null_text.py:290-311."""


class AttentionReweight(AttentionControlEdit, _c.AttentionReweight):
    """null_text.py:314-337."""


for _cls in (AttentionReplace, AttentionRefine, AttentionReweight):
    _cls._P2P_LIB = True


def get_equalizer(text: str, word_select: Union[int, Tuple[int, ...]],
                  values: Union[List[float], Tuple[float, ...]], tokenizer=None):
    """null_text.py:340-349: a single row, one value per selected word."""
    tokenizer = tokenizer or get_tokenizer()
    if type(word_select) is int or type(word_select) is str:
        word_select = (word_select,)
    eq = torch.ones(1, MAX_NUM_WORDS)
    for word, val in zip(word_select, values):
        eq[:, get_word_inds(text, word, tokenizer)] = val
    return eq


def make_controller(prompts: List[str], is_replace_controller: bool, cross_replace_steps: Dict[str, float],
                    self_replace_steps: float, blend_words=None, equilizer_params=None,
                    tokenizer=None, device=None) -> AttentionControlEdit:
    """null_text.py:369-401 (with its ``blend_word`` NameError fixed)."""
    lb = None if blend_words is None else LocalBlend(prompts, blend_words, tokenizer=tokenizer, device=device)
    kw = dict(cross_replace_steps=cross_replace_steps, self_replace_steps=self_replace_steps, local_blend=lb,
              tokenizer=tokenizer, device=device)
    cls = AttentionReplace if is_replace_controller else AttentionRefine
    controller = cls(prompts, NUM_DDIM_STEPS, **kw)
    if equilizer_params is not None:
        eq = get_equalizer(prompts[1], equilizer_params["words"], equilizer_params["values"], tokenizer)
        controller = AttentionReweight(prompts, NUM_DDIM_STEPS, equalizer=eq, controller=controller, **kw)
    return controller


# ============================================================================ null-text inversion
def load_512(image_path, left=0, right=0, top=0, bottom=0):
    """null_text.py:447-466: crop by the offsets, centre-square, resize to 512 (needs PIL)."""
    import numpy as np
    from PIL import Image
    image = np.array(Image.open(image_path))[:, :, :3] if isinstance(image_path, str) else image_path
    h, w, _ = image.shape
    left = min(left, w - 1)
    right = min(right, w - left - 1)
    top = min(top, h - left - 1)
    bottom = min(bottom, h - top - 1)
    image = image[top:h - bottom, left:w - right]
    h, w, _ = image.shape
    if h < w:
        image = image[:, (w - h) // 2:(w - h) // 2 + h]
    elif w < h:
        image = image[(h - w) // 2:(h - w) // 2 + w]
    return np.array(Image.fromarray(image).resize((512, 512)))


class NullInversion:
    """null_text.py:469-628 on this library's kernels.

    DDIM inversion of the image latent with the conditional U-Net (``ddim_loop``), then, per
    step, up to ``num_inner_steps`` Adam updates of the null (unconditional) embedding so that
    the guided DDIM step lands on the inverted trajectory (``null_optimization``).  Every update
    back-propagates through all 32 patched attentions: the hook is installed with no controller
    (null_text.py:610), whose plain path is differentiable on the HIP kernels
    (attention._AttentionFn: p2p_attn_fwd_lse / p2p_attn_bwd).  ``invert`` also takes the image
    latent itself ([1, 4, H/8, W/8], the form the reference's ``image2latent`` passes through):
    the synthetic pipeline has no VAE."""

    def __init__(self, model, num_ddim_steps: int = NUM_DDIM_STEPS, guidance_scale: float = GUIDANCE_SCALE,
                 use_graphs: bool = True):
        self.model = model
        self.tokenizer = model.tokenizer
        self.num_ddim_steps = num_ddim_steps
        self.guidance_scale = guidance_scale
        self.use_graphs = use_graphs
        self.model.scheduler.set_timesteps(num_ddim_steps)
        self.prompt = None
        self.context = None

    @property
    def scheduler(self):
        return self.model.scheduler

    def prev_step(self, model_output, timestep, sample):
        return self.scheduler.prev_step(model_output, timestep, sample)

    def next_step(self, model_output, timestep, sample):
        return self.scheduler.next_step(model_output, timestep, sample)

    def get_noise_pred_single(self, latents, t, context):
        return self.model.unet(latents, t, encoder_hidden_states=context)["sample"]

    def get_noise_pred(self, latents, t, is_forward=True, context=None):
        context = self.context if context is None else context
        eps = self.model.unet(torch.cat([latents] * 2), t, encoder_hidden_states=context)["sample"]
        eps_u, eps_c = eps.chunk(2)
        g = 1 if is_forward else self.guidance_scale
        eps = eps_u + g * (eps_c - eps_u)
        return self.next_step(eps, t, latents) if is_forward else self.prev_step(eps, t, latents)

    @torch.no_grad()
    def latent2image(self, latents, return_type="np"):
        vae = getattr(self.model, "vae", None)
        if vae is None:
            return None
        image = vae.decode(1 / 0.18215 * latents.detach())["sample"]
        if return_type == "np":
            image = (image / 2 + 0.5).clamp(0, 1).cpu().permute(0, 2, 3, 1).numpy()[0]
            image = (image * 255).astype("uint8")
        return image

    @torch.no_grad()
    def image2latent(self, image):
        if torch.is_tensor(image) and image.dim() == 4:
            return image.to(self.model.device)
        vae = getattr(self.model, "vae", None)
        if vae is None:
            raise ValueError("this pipeline has no VAE: pass the image latent [1, 4, H/8, W/8]")
        import numpy as np
        x = torch.from_numpy(np.asarray(image)).float() / 127.5 - 1
        x = x.permute(2, 0, 1).unsqueeze(0).to(self.model.device)
        return vae.encode(x)["latent_dist"].mean * 0.18215

    @torch.no_grad()
    def init_prompt(self, prompt: str):
        def encode(texts):
            ids = self.tokenizer(texts, padding="max_length", max_length=self.tokenizer.model_max_length,
                                 truncation=True, return_tensors="pt").input_ids
            return self.model.text_encoder(ids.to(self.model.device))[0]
        self.context = torch.cat([encode([""]), encode([prompt])])
        self.prompt = prompt

    @torch.no_grad()
    def ddim_loop(self, latent):
        cond = self.context.chunk(2)[1]
        trajectory = [latent]
        latent = latent.clone().detach()
        ts = self.scheduler.timesteps
        for i in range(self.num_ddim_steps):
            t = ts[len(ts) - i - 1]
            latent = self.next_step(self.get_noise_pred_single(latent, t, cond), t, latent)
            trajectory.append(latent)
        return trajectory

    @torch.no_grad()
    def ddim_inversion(self, image):
        latent = self.image2latent(image)
        return self.latent2image(latent), self.ddim_loop(latent)

    def null_optimization(self, latents, num_inner_steps, epsilon):
        import torch.nn.functional as F
        if self.use_graphs and latents[-1].is_cuda and hasattr(self.scheduler, "prev_coeffs"):
            return self._null_optimization_graphed(latents, num_inner_steps, epsilon)
        uncond, cond = self.context.chunk(2)
        per_step = []
        latent_cur = latents[-1]
        for i in range(self.num_ddim_steps):
            uncond = uncond.clone().detach().requires_grad_(True)
            opt = torch.optim.Adam([uncond], lr=1e-2 * (1.0 - i / 100.0))
            latent_prev = latents[len(latents) - i - 2]
            t = self.scheduler.timesteps[i]
            with torch.no_grad():
                eps_c = self.get_noise_pred_single(latent_cur, t, cond)
            for _ in range(num_inner_steps):
                eps_u = self.get_noise_pred_single(latent_cur, t, uncond)
                eps = eps_u + self.guidance_scale * (eps_c - eps_u)
                loss = F.mse_loss(self.prev_step(eps, t, latent_cur), latent_prev)
                opt.zero_grad()
                loss.backward()
                opt.step()
                if loss.item() < epsilon + i * 2e-5:
                    break
            per_step.append(uncond[:1].detach())
            with torch.no_grad():
                latent_cur = self.get_noise_pred(latent_cur, t, False, torch.cat([uncond, cond]))
        return per_step

    def _null_optimization_graphed(self, latents, num_inner_steps, epsilon):
        """null_optimization with each inner step (null_text.py:587-598: U-Net forward with the null
        embedding as the only leaf, guided DDIM step, MSE, backward, Adam update) replayed from one
        captured HIP graph.  The batch-1 step is host-bound eagerly (~40 ms of Python/launch work
        for ~1500 kernels); the graph is captured once per inversion, and per DDIM step only its
        inputs, the parameter, the Adam state and the learning rate are refilled in place.  The
        early stop (null_text.py:597) still reads the loss after every step, as the reference."""
        uncond, cond = self.context.chunk(2)
        unet = self.model.unet
        t0 = self.scheduler.timesteps[0]
        step = _GraphedNullStep(self, latents[-1], uncond)
        fwd_c = _GraphedForward(unet, latents[-1], cond, t0)                               # eps_c
        fwd_cfg = _GraphedForward(unet, torch.cat([latents[-1]] * 2), torch.cat([uncond, cond]), t0)
        per_step = []
        self.inner_steps_run = 0
        latent_cur = latents[-1]
        for i in range(self.num_ddim_steps):
            latent_prev = latents[len(latents) - i - 2]
            t = self.scheduler.timesteps[i]
            eps_c = fwd_c(latent_cur, t, cond)
            step.reset(uncond, 1e-2 * (1.0 - i / 100.0), latent_cur, eps_c, latent_prev, t)
            for _ in range(num_inner_steps):
                step.graph.replay()
                self.inner_steps_run += 1
                if step.loss.item() < epsilon + i * 2e-5:
                    break
            uncond = step.param.detach().clone()
            per_step.append(uncond[:1])
            with torch.no_grad():                       # get_noise_pred(is_forward=False), graphed U-Net
                eps = fwd_cfg(torch.cat([latent_cur] * 2), t, torch.cat([uncond, cond]))
                eps_u, eps_cc = eps.chunk(2)
                latent_cur = self.prev_step(eps_u + self.guidance_scale * (eps_cc - eps_u), t, latent_cur)
        return per_step

    def invert(self, image, prompt: str, offsets=(0, 0, 0, 0), num_inner_steps=10, early_stop_epsilon=1e-5,
               verbose=False):
        from . import ptp_utils
        self.init_prompt(prompt)
        ptp_utils.register_attention_control(self.model, None)
        image_gt = load_512(image, *offsets) if isinstance(image, str) else image
        if verbose:
            print("DDIM inversion...")
        image_rec, ddim_latents = self.ddim_inversion(image_gt)
        if verbose:
            print("Null-text optimization...")
        uncond_embeddings = self.null_optimization(ddim_latents, num_inner_steps, early_stop_epsilon)
        return (image_gt, image_rec), ddim_latents[-1], uncond_embeddings


class _GraphedForward:
    """A no-grad U-Net call on fixed shapes captured as a HIP graph; __call__ refills the static
    latent / timestep / context and replays (the output tensor is reused by the next replay)."""

    def __init__(self, unet, x, ctx, t):
        dev = x.device
        self.x = x.detach().clone()
        self.ctx = ctx.detach().clone()
        self.t = torch.full((1,), int(t), dtype=torch.int64, device=dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.no_grad():
            with torch.cuda.stream(side):
                for _ in range(2):
                    unet(self.x, self.t, encoder_hidden_states=self.ctx)
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = unet(self.x, self.t, encoder_hidden_states=self.ctx)["sample"]

    @torch.no_grad()
    def __call__(self, x, t, ctx):
        self.x.copy_(x)
        self.ctx.copy_(ctx)
        self.t.fill_(int(t))
        self.graph.replay()
        return self.out


class _GraphedNullStep:
    """One null-text Adam step captured as a HIP graph (NullInversion._null_optimization_graphed).
    Static inputs: the latent, eps_c, the target latent, the timestep and the four DDIM
    coefficients of prev_step (ddim.DDIMScheduler.prev_coeffs: sqrt(1 - a_t), sqrt(a_t),
    sqrt(a_prev), sqrt(1 - a_prev)); the parameter and the capturable Adam state are updated in
    place by every replay."""

    def __init__(self, inv, latent, uncond):
        import torch.nn.functional as F
        dev = latent.device
        self.inv = inv
        self.x = latent.detach().clone()
        self.eps_c = torch.zeros_like(self.x)
        self.target = torch.zeros_like(self.x)
        self.t = torch.zeros(1, dtype=torch.int64, device=dev)
        self.coef = torch.zeros(4, dtype=torch.float32, device=dev)
        self.param = uncond.detach().clone().requires_grad_(True)
        self.lr = torch.tensor(1e-2, dtype=torch.float32, device=dev)
        self.opt = torch.optim.Adam([self.param], lr=self.lr, capturable=True)
        g = inv.guidance_scale
        unet = inv.model.unet

        def body():
            self.opt.zero_grad(set_to_none=False)
            eps_u = unet(self.x, self.t, encoder_hidden_states=self.param)["sample"]
            eps = eps_u + g * (self.eps_c - eps_u)
            x0 = (self.x - self.coef[0] * eps) / self.coef[1]
            prev = self.coef[2] * x0 + self.coef[3] * eps
            loss = F.mse_loss(prev, self.target)
            loss.backward()
            self.opt.step()
            return loss

        # warm-up on a side stream (autograd buffers, Adam state, allocator), then capture
        self.t.fill_(int(inv.scheduler.timesteps[0]))
        self.coef.copy_(self._coeffs(inv.scheduler.timesteps[0]))
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):
                body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = body()

    def _coeffs(self, t):
        c = self.inv.scheduler.prev_coeffs(t)        # (sqrt_beta_t, sqrt_alpha_t, sqrt_alpha_prev, sqrt_1m_alpha_prev)
        return torch.tensor([float(x) for x in c], dtype=torch.float32)

    @torch.no_grad()
    def reset(self, uncond, lr, latent, eps_c, target, t):
        """A fresh Adam on a fresh copy of the null embedding (null_text.py:582-584)."""
        self.param.copy_(uncond)
        for st in self.opt.state.values():
            for key in ("step", "exp_avg", "exp_avg_sq"):
                st[key].zero_()
        self.lr.fill_(lr)
        self.x.copy_(latent)
        self.eps_c.copy_(eps_c)
        self.target.copy_(target)
        self.t.fill_(int(t))
        self.coef.copy_(self._coeffs(t))
