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

    def step_mask(self, attention_store, size):
        """What __call__ does to its counter, returning the mask it would blend with (or None
        before start_blend) -- the fused latent-step protocol."""
        self.counter += 1
        if self.counter > self.start_blend:
            self._size = tuple(size)
            sub = self._sub_flat if self.substruct_layers is not None else None
            return _c.fused_blend_mask(attention_store, self._alpha_flat, sub, self.th[0], self.th[1], size)
        return None

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
