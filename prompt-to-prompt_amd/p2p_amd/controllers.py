"""Prompt-to-Prompt attention controllers -- the reference API, fused underneath.

Public surface of ``main.py:33-307`` (same class names, constructor arguments, attributes
and ``__call__`` / ``forward`` / ``step_callback`` / ``between_steps`` / ``reset`` /
``get_average_attention`` protocol).  The difference is underneath: when the patched
``CrossAttention.forward`` (ptp_utils.register_attention_control) finds one of these
controllers, it calls :meth:`AttentionControl.attention`, which launches ONE HIP kernel per
call that computes the attention with the controller's edit and store fused in:

* self-attention: flash kernel; source-map injection as a batch index remap;
* cross-attention: exact-softmax kernel; Replace / Refine / Reweight as a device edit
  program (programs.py) applied between softmax and PV;
* AttentionStore: probabilities written (step 0) or added (later steps) to the running-sum
  tensors in the kernel epilogue, only for the maps the reference keeps (P <= 32**2).

A subclass that overrides any method the fused kernel encodes (``forward``,
``replace_cross_attention``, ``replace_self_attention``, ``__call__``) gets the reference
protocol instead: the probabilities are materialised by a HIP kernel, handed to
``controller(attn, is_cross, place_in_unet)`` and multiplied by V by a second HIP kernel.
"""
from __future__ import annotations

import abc
from collections import defaultdict
from typing import Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from . import _hip
from . import config
from . import programs
from . import seq_aligner
from .attention import materialized_attention, plain_attention
from .ptp_words import get_time_words_attention_alpha, get_word_inds
from .tokenizer import default_tokenizer

NUM_DIFFUSION_STEPS = 100   # main.py:19
GUIDANCE_SCALE = 7.5        # main.py:20
MAX_NUM_WORDS = 77          # main.py:21
MAX_STORED_QUERIES = 32 ** 2  # main.py:131

_tokenizer = None


def set_tokenizer(tokenizer):
    """The reference reads a module-global ``tokenizer`` (main.py:30); this sets ours."""
    global _tokenizer
    _tokenizer = tokenizer


def get_tokenizer():
    return _tokenizer if _tokenizer is not None else default_tokenizer()


def default_device() -> torch.device:
    return torch.device("cuda:0") if torch.cuda.is_available() else torch.device("cpu")


def _low_resource() -> bool:
    return bool(config.LOW_RESOURCE)


class NotFusable(Exception):
    """Raised while planning a fused call that the kernels cannot express."""


# ============================================================================ LocalBlend
def fused_local_blend(x_t, attention_store, alpha_flat, sub_flat, th_pool, th_sub):
    """LocalBlend on the running-sum store with the HIP blend kernels (returns a new x_t)."""
    maps = list(attention_store["down_cross"][2:4]) + list(attention_store["up_cross"][:3])
    B = alpha_flat.shape[0]
    if len(maps) != 5:
        raise ValueError(f"LocalBlend needs 2 down and 3 up 16x16 cross maps, store has {len(maps)}")
    heads = maps[0].shape[0] // B
    maps = [m if (m.dtype == torch.float32 and m.is_contiguous()) else m.float().contiguous() for m in maps]
    out = x_t.to(torch.float32).contiguous().clone()
    ws = torch.empty(B * 2 * len(maps) * heads * maps[0].shape[1], dtype=torch.float32, device=out.device)
    _hip.localblend(maps, heads, alpha_flat, sub_flat, th_pool, th_sub, out, ws)
    return out.to(x_t.dtype)


class FoldedBlendMask:
    """One prompt group's LocalBlend mask in the form it is built from: the running word sums
    [B, 2, lh, res^2] that the cross-attention store epilogue folded (AttentionControlEdit.
    _blend_fold).  p2p_latent_step builds the mask from them inside the latent-update launch --
    LocalBlend and the CFG/DDIM step are one kernel per denoising step (null_text.py:41-70,
    ptp_utils.py:72-75).  materialize() builds the same mask as a uint8 [B, H, W] tensor with
    p2p_localblend (mixed prompt-group batches, tests)."""

    def __init__(self, maps, heads, alpha_flat, sub_flat, th_pool, th_sub, size, sums):
        self._maps, self._heads, self._alpha, self._sub = maps, heads, alpha_flat, sub_flat
        self.th_pool, self.th_sub, self.size, self.sums = float(th_pool), float(th_sub), tuple(size), sums

    def latent_entry(self):
        """The per-group entry of _hip.latent_step(blend=...)."""
        return self.sums, self.th_pool, self.th_sub, self._sub is not None

    def materialize(self) -> torch.Tensor:
        mask = torch.empty(self._alpha.shape[0], *self.size, dtype=torch.uint8, device=self.sums.device)
        _hip.localblend(self._maps, self._heads, self._alpha, self._sub, self.th_pool, self.th_sub, None, self.sums,
                        mask_out=mask, word_sums_ready=True)
        return mask


def as_mask(m):
    """A step mask as a uint8 tensor (materialising a FoldedBlendMask), or None."""
    return m.materialize() if isinstance(m, FoldedBlendMask) else m


def group_mask_tensor(masks, B, size):
    """Per-group step masks (None = the group does not blend) as the mask-reading latent step's
    (mask [G*B, H, W] uint8, group size, groups that blend [G] uint8) triple."""
    masks = [as_mask(mk) for mk in masks]
    dev = next(mk for mk in masks if mk is not None).device
    out = torch.zeros(len(masks) * B, *size, dtype=torch.uint8, device=dev)
    blend = torch.zeros(len(masks), dtype=torch.uint8)
    for g, mk in enumerate(masks):
        if mk is not None:
            out[g * B:(g + 1) * B] = mk
            blend[g] = 1
    return out, B, blend.to(dev)


def fused_blend_mask(attention_store, alpha_flat, sub_flat, th_pool, th_sub, size, folded=None):
    """LocalBlend's final mask [B, H, W] (uint8) only; the latent blend itself then runs inside
    p2p_latent_step together with the CFG combine and the DDIM step.  ``folded``: the running word
    sums [B, 2, 5 * heads, 256] that the cross-attention store epilogue accumulated
    (AttentionControlEdit._blend_fold) -- then the 12.6 MB of maps are not re-read, and the mask
    is returned as a FoldedBlendMask that p2p_latent_step builds in the same launch."""
    maps = list(attention_store["down_cross"][2:4]) + list(attention_store["up_cross"][:3])
    B = alpha_flat.shape[0]
    if len(maps) != 5:
        raise ValueError(f"LocalBlend needs 2 down and 3 up 16x16 cross maps, store has {len(maps)}")
    heads = maps[0].shape[0] // B
    dev = maps[0].device
    if folded is not None:
        return FoldedBlendMask(maps, heads, alpha_flat, sub_flat, th_pool, th_sub, size, folded)
    mask = torch.empty(B, *size, dtype=torch.uint8, device=dev)
    maps = [m if (m.dtype == torch.float32 and m.is_contiguous()) else m.float().contiguous() for m in maps]
    ws = torch.empty(B * 2 * len(maps) * heads * maps[0].shape[1], dtype=torch.float32, device=dev)
    _hip.localblend(maps, heads, alpha_flat, sub_flat, th_pool, th_sub, None, ws, mask_out=mask)
    return mask


def _owned(obj, name) -> bool:
    """True when ``name`` resolves to a method this library defines (not a user override)."""
    for owner in type(obj).__mro__:
        if name in owner.__dict__:
            return bool(owner.__dict__.get("_P2P_LIB", False))
    return False


def _word_alpha_layers(prompts, words, tokenizer, n_words=MAX_NUM_WORDS):
    a = torch.zeros(len(prompts), 1, 1, 1, 1, n_words)
    for i, (prompt, ws) in enumerate(zip(prompts, words)):
        for word in ([ws] if type(ws) is str else ws):
            a[i, :, :, :, :, get_word_inds(prompt, word, tokenizer)] = 1
    return a


class LocalBlend:
    """main.py:33-66.  Valid for two prompts only, as in the reference (its mask
    ``mask[:1] + mask[1:]`` does not broadcast for more); use null_text.LocalBlend for B > 2."""

    def __call__(self, x_t, attention_store):
        if self.alpha_layers.shape[0] != 2:
            raise ValueError("main-form LocalBlend broadcasts only for 2 prompts (see null_text.LocalBlend)")
        return fused_local_blend(x_t, attention_store, self._alpha_flat, None, self.threshold, self.threshold)

    def step_mask(self, attention_store, size, folded=None):
        """The blend mask __call__ would apply this step (fused latent-step protocol)."""
        if self.alpha_layers.shape[0] != 2:
            raise ValueError("main-form LocalBlend broadcasts only for 2 prompts (see null_text.LocalBlend)")
        return fused_blend_mask(attention_store, self._alpha_flat, None, self.threshold, self.threshold, size,
                                folded)

    def _fold_tables(self):
        """(alpha [B, W], substruct [B, W] or None) the store epilogue folds the word sums with."""
        return self._alpha_flat, None

    def __init__(self, prompts: List[str], words, threshold=.3, tokenizer=None, device=None):
        tokenizer = tokenizer or get_tokenizer()
        device = device or default_device()
        self.alpha_layers = _word_alpha_layers(prompts, words, tokenizer).to(device)
        self._alpha_flat = self.alpha_layers.reshape(len(prompts), -1).contiguous()
        self.threshold = threshold


LocalBlend._P2P_LIB = True


# ============================================================================ controllers
class AttentionControl(abc.ABC):
    """main.py:69-107 -- step/layer counters and the cond-half dispatch."""

    _NATIVE = ("__call__",)

    def step_callback(self, x_t):
        return x_t

    def fused_step_mask(self):
        """Fused latent-step protocol (ptp_utils.diffusion_step): (True, mask_fn) when this
        step's step_callback is this library's own -- mask_fn(size) then has the callback's
        side effects and returns the LocalBlend mask or None -- else (False, None)."""
        if not _owned(self, "step_callback"):
            return False, None
        return True, self._step_mask_fn()

    def _step_mask_fn(self):
        return None

    def between_steps(self):
        return

    @property
    def num_uncond_att_layers(self):
        return self.num_att_layers if _low_resource() else 0

    @abc.abstractmethod
    def forward(self, attn, is_cross: bool, place_in_unet: str):
        raise NotImplementedError

    def __call__(self, attn, is_cross: bool, place_in_unet: str):
        if self.cur_att_layer >= self.num_uncond_att_layers:
            if _low_resource():
                attn = self.forward(attn, is_cross, place_in_unet)
            else:
                half = attn.shape[0] // 2
                attn[half:] = self.forward(attn[half:], is_cross, place_in_unet)
        self._advance_layer()
        return attn

    def _advance_layer(self):
        self.cur_att_layer += 1
        if self.cur_att_layer == self.num_att_layers + self.num_uncond_att_layers:
            self.cur_att_layer = 0
            self.cur_step += 1
            self.between_steps()

    def reset(self):
        self.cur_step = 0
        self.cur_att_layer = 0

    def __init__(self):
        self.cur_step = 0
        self.num_att_layers = -1
        self.cur_att_layer = 0

    # ------------------------------------------------------------------ fused protocol
    def fused_supported(self) -> bool:
        """True when every method the fused kernels encode is this library's own."""
        cls = type(self)
        names = set()
        for owner in cls.__mro__:
            names.update(owner.__dict__.get("_NATIVE", ()))
        for name in names:
            # the class that resolves `name` must be one of ours
            for owner in cls.__mro__:
                if name in owner.__dict__:
                    if not owner.__dict__.get("_P2P_LIB", False):
                        return False
                    break
        return True

    def _fused_forward(self, q, k, v, heads, scale, is_cross, place_in_unet):
        raise NotFusable

    def attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask=None):
        """Called by the patched CrossAttention.forward with the projections q, k, v."""
        if mask is None and self.fused_supported():
            try:
                if self.cur_att_layer >= self.num_uncond_att_layers:
                    out = self._fused_forward(q, k, v, heads, scale, is_cross, place_in_unet)
                else:
                    out = plain_attention(q, k, v, heads, scale)
                self._advance_layer()
                return out
            except NotFusable:
                pass
        return materialized_attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask)

    def _cond_start(self, n_batch: int) -> int:
        return 0 if _low_resource() else n_batch // 2


AttentionControl._P2P_LIB = True


class EmptyControl(AttentionControl):
    """main.py:110-113."""

    _NATIVE = ("forward",)

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        return attn

    def _fused_forward(self, q, k, v, heads, scale, is_cross, place_in_unet):
        return plain_attention(q, k, v, heads, scale)


EmptyControl._P2P_LIB = True


class AttentionStore(AttentionControl):
    """main.py:116-159.  ``store_self_maps = False`` keeps only the cross maps (the ones
    LocalBlend and ``show_cross_attention`` read); the default matches the reference."""

    _NATIVE = ("forward", "between_steps")
    store_self_maps = True

    @staticmethod
    def get_empty_store():
        return {"down_cross": [], "mid_cross": [], "up_cross": [],
                "down_self": [], "mid_self": [], "up_self": []}

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        key = f"{place_in_unet}_{'cross' if is_cross else 'self'}"
        if attn.shape[1] <= MAX_STORED_QUERIES:
            self.step_store[key].append(attn)
        return attn

    def between_steps(self):
        if len(self.attention_store) == 0:
            self.attention_store = self.step_store
        else:
            # fused calls already added their maps in the kernel epilogue; only maps handed
            # over through the materialised protocol are still pending here
            for key, items in self.step_store.items():
                for i, item in enumerate(items):
                    self.attention_store[key][i] += item
        self.step_store = self.get_empty_store()
        self._fused_calls = defaultdict(int)

    def get_average_attention(self):
        def avg(item):
            if item.is_cuda and item.dtype == torch.float32 and item.is_contiguous():
                return _hip.store_scale(item, float(self.cur_step))
            return item / self.cur_step
        return {key: [avg(item) for item in self.attention_store[key]] for key in self.attention_store}

    def reset(self):
        super().reset()
        self.step_store = self.get_empty_store()
        self.attention_store = {}
        self._fused_calls = defaultdict(int)

    def __init__(self):
        super().__init__()
        self.step_store = self.get_empty_store()
        self.attention_store = {}
        self._fused_calls = defaultdict(int)

    # ------------------------------------------------------------------ fused store
    def _store_target(self, is_cross, place_in_unet, n_cond, heads, P, K, device):
        """Running-sum tensor this call's maps go to, and whether to add or overwrite."""
        if P > MAX_STORED_QUERIES or (not is_cross and not self.store_self_maps):
            return None, False
        key = f"{place_in_unet}_{'cross' if is_cross else 'self'}"
        idx = self._fused_calls[key]
        self._fused_calls[key] = idx + 1
        self._last_store_key = (key, idx)
        if len(self.attention_store) == 0:
            t = torch.empty(n_cond * heads, P, K, dtype=torch.float32, device=device)
            self.step_store[key].append(t)
            return t, False
        return self.attention_store[key][idx], True

    def _slots(self, n_batch, n0, heads, store):
        if store is None:
            return None
        return [-1] * n0 + [(n - n0) * heads for n in range(n0, n_batch)]

    def _fused_forward(self, q, k, v, heads, scale, is_cross, place_in_unet):
        N, P, K = q.shape[0], q.shape[1], k.shape[1]
        n0 = self._cond_start(N)
        store, acc = self._store_target(is_cross, place_in_unet, N - n0, heads, P, K, q.device)
        slots = self._slots(N, n0, heads, store)
        out = torch.empty_like(q)
        if is_cross and K <= _hip.MAX_KEYS_CROSS:
            groups = [(0, N, None, None)]
            _hip.cross_attn(q, k, v, out, heads, scale, groups, compute=config.COMPUTE, store=store,
                            store_slot=slots, accumulate=acc)
        else:
            _hip.self_attn(q, k, v, out, heads, scale, compute=config.COMPUTE, store=store,
                           store_slot=slots, accumulate=acc)
        return out


AttentionStore._P2P_LIB = True


class AttentionControlEdit(AttentionStore, abc.ABC):
    """main.py:162-212."""

    _NATIVE = ("forward", "replace_self_attention", "_replace_self")
    SELF_REPLACE_MAX_KEYS = 16 ** 2   # main.py:170 (null_text.py:225 uses 32 ** 2)

    def step_callback(self, x_t):
        if self.local_blend is not None:
            x_t = self.local_blend(x_t, self.attention_store)
        return x_t

    def _step_mask_fn(self):
        lb = self.local_blend
        if lb is None:
            return None
        if not (_owned(lb, "__call__") and hasattr(lb, "step_mask")):
            raise NotFusable
        return lambda size: lb.step_mask(self.attention_store, size,
                                         folded=self._blend_sums if self._blend_valid else None)

    # LocalBlend's word reduction folded into the cross-attention store epilogue: the five 16x16
    # cross layers it reads (main.py:37-38, down_cross[2:4] + up_cross[:3]) get their running word
    # sums accumulated by the kernel that writes their maps, so the blend reads ~0.3 MB instead
    # of the 12.6 MB of maps every step.  Valid only while EVERY step folded all five layers.
    BLEND_SLOTS = {("down_cross", 2): 0, ("down_cross", 3): 1, ("up_cross", 0): 2, ("up_cross", 1): 3,
                   ("up_cross", 2): 4}
    # The fold sums each step's word sums (sum over steps of sum over words) where the reference
    # takes the word sums of the summed maps (main.py:37-44): equal in exact arithmetic, a
    # different f32 summation order in practice, so a pixel sitting on the threshold can flip
    # (tests/test_gpu_blend_fold.py pins the agreement).  False = strict parity: the blend reads
    # the stored maps as the reference does.
    fold_local_blend = True

    def _blend_fold(self, key_idx, P, K, heads, device):
        """The p2p_group.blend_* tuple for this stored cross layer, or None."""
        lb = self.local_blend
        slot = self.BLEND_SLOTS.get(key_idx)
        if not self.fold_local_blend or slot is None or lb is None or P != 256 or not (_owned(lb, "__call__") and hasattr(lb, "_fold_tables")):
            return None
        alpha, sub = lb._fold_tables()
        if alpha.shape != (self.batch_size, K) or alpha.device != device:
            return None
        lh = len(self.BLEND_SLOTS) * heads
        if len(self.attention_store) == 0 and slot == 0:
            self._blend_sums = torch.empty(self.batch_size, 2, lh, P, dtype=torch.float32, device=device)
            self._blend_valid = False
            self._blend_step = set()
        if self._blend_sums is None or self._blend_sums.shape != (self.batch_size, 2, lh, P):
            return None
        self._blend_step.add(slot)
        return self._blend_sums, alpha, sub, slot * heads, lh

    def between_steps(self):
        # a step in which some blend layer did not fold (materialised protocol, a new run) ends
        # the folded sums' validity until the next reset
        first = len(self.attention_store) == 0
        complete = self._blend_sums is not None and len(self._blend_step) == len(self.BLEND_SLOTS)
        self._blend_valid = complete and (first or self._blend_valid)
        self._blend_step = set()
        super().between_steps()

    def reset(self):
        super().reset()
        self._blend_sums, self._blend_valid, self._blend_step = None, False, set()

    def fused_step_mask(self):
        try:
            return super().fused_step_mask()
        except NotFusable:
            return False, None

    def replace_self_attention(self, attn_base, att_replace):
        if att_replace.shape[2] <= self.SELF_REPLACE_MAX_KEYS:
            return attn_base.unsqueeze(0).expand(att_replace.shape[0], *attn_base.shape)
        return att_replace

    @abc.abstractmethod
    def replace_cross_attention(self, attn_base, att_replace):
        raise NotImplementedError

    def _in_self_window(self) -> bool:
        return self.num_self_replace[0] <= self.cur_step < self.num_self_replace[1]

    def _replace_self(self, attn_base, att_replace, place_in_unet):
        return self.replace_self_attention(attn_base, att_replace)

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        """Reference protocol on a materialised [B*H, P, K] tensor (main.py:180-197)."""
        AttentionStore.forward(self, attn, is_cross, place_in_unet)
        if not (is_cross or self._in_self_window()):
            return attn
        per_prompt = attn.reshape(self.batch_size, attn.shape[0] // self.batch_size, *attn.shape[1:])
        base, edits = per_prompt[0], per_prompt[1:]
        if is_cross:
            a = self.cross_replace_alpha[self.cur_step]
            per_prompt[1:] = self.replace_cross_attention(base, edits) * a + (1 - a) * edits
        else:
            per_prompt[1:] = self._replace_self(base, edits, place_in_unet)
        return per_prompt.reshape(attn.shape[0], *attn.shape[1:])

    def __init__(self, prompts, num_steps: int,
                 cross_replace_steps: Union[float, Tuple[float, float], Dict[str, Tuple[float, float]]],
                 self_replace_steps: Union[float, Tuple[float, float]],
                 local_blend: Optional[LocalBlend], tokenizer=None, device=None):
        super().__init__()
        self.tokenizer = tokenizer or get_tokenizer()
        self.device = device or default_device()
        self.batch_size = len(prompts)
        self.cross_replace_alpha = get_time_words_attention_alpha(
            prompts, num_steps, cross_replace_steps, self.tokenizer).to(self.device)
        if type(self_replace_steps) is float:
            self_replace_steps = 0, self_replace_steps
        self.num_self_replace = int(num_steps * self_replace_steps[0]), int(num_steps * self_replace_steps[1])
        self.local_blend = local_blend
        self._program_cache = {}
        self._program_host = None
        self._alpha_host = None
        self._step_cache = {}
        self._blend_sums, self._blend_valid, self._blend_step = None, False, set()

    # ------------------------------------------------------------------ fused edits
    def _edit_program(self) -> programs.EditProgram:
        raise NotFusable

    def _device_program(self, device):
        key = str(device)
        if key not in self._program_cache:
            try:
                host = self._edit_program()
                self._program_cache[key] = host.to_device(device)
                self._program_host = host
            except ValueError as err:      # beyond the program tables: materialised protocol
                raise NotFusable from err
        return self._program_cache[key]

    def _cross_step(self, device, K):
        """The cross-attention edit of this step as (program or None, p2p_group hint flags), from
        the host copy of cross_replace_alpha[cur_step] (main.py:189) and the program's c_rep / post:
        with B = alpha post and A = alpha post c_rep + 1 - alpha on every word of every edit,
          * B = 0 and A = 1 everywhere (past cross_replace_steps): P' = R * 0 + P_e = P_e exactly,
            the group runs unedited (no program: the kernels load no mapper, no source rows);
          * A = 0 everywhere (a Replace / Reweight step inside the window): P' = R B, the edits'
            own softmax, Q and K are dead -- GROUP_F_R_ONLY.
        Decided once per step (the alpha table is copied to the host once)."""
        prog = self._device_program(device)
        alpha = self.cross_replace_alpha
        # (the tensor itself, its version, host copy): identity, not id().  A tensor made under
        # torch.inference_mode() has no version counter: its storage address stands in for it
        version = ("ptr", alpha.data_ptr()) if alpha.is_inference() else alpha._version
        held = self._alpha_host
        if held is None or held[0] is not alpha or held[1] != version:
            held = self._alpha_host = (alpha, version, alpha.detach().to("cpu", torch.float64).numpy())
            self._step_cache = {}
        key = (self.cur_step, K)
        hit = self._step_cache.get(key)
        if hit is not None:
            return (None if hit[0] else prog), hit[1]
        host = self._program_host
        a = held[2][self.cur_step].reshape(host.n_edits, -1)[:, :K]
        post = host.post[:, :K].astype(np.float64)
        crep = host.c_rep[:, :K].astype(np.float64)
        B = a * post
        A = B * crep + (1.0 - a)
        plain = bool(np.all(B == 0.0) and np.all(A == 1.0))
        hints = _hip.GROUP_F_R_ONLY if np.all(A == 0.0) else 0
        self._step_cache[key] = (plain, hints)
        return (None if plain else prog), hints

    def _fused_forward(self, q, k, v, heads, scale, is_cross, place_in_unet):
        N, P, K = q.shape[0], q.shape[1], k.shape[1]
        n0 = self._cond_start(N)
        n_cond = N - n0
        if n_cond != self.batch_size:
            raise ValueError(f"controller built for {self.batch_size} prompts got a batch of {n_cond}")
        if is_cross:
            alpha = self.cross_replace_alpha[self.cur_step]
            if K > _hip.MAX_KEYS_CROSS or alpha.shape[-1] != K or alpha.device != q.device:
                raise NotFusable
            prog, hints = self._cross_step(q.device, K)
        store, acc = self._store_target(is_cross, place_in_unet, n_cond, heads, P, K, q.device)
        slots = self._slots(N, n0, heads, store)
        out = torch.empty_like(q)
        if is_cross:
            blend = self._blend_fold(self._last_store_key, P, K, heads, q.device) if store is not None else None
            # the uncond rows ("" prompts) share their K / V: staged once per workgroup (SHARED_KV)
            groups = (([(0, n0, None, None, None, _hip.shared_kv_hint(k, v, 0, n0))] if n0 else [])
                      + [(n0, n_cond, prog, alpha.contiguous(), blend, hints)])
            _hip.cross_attn(q, k, v, out, heads, scale, groups, compute=config.COMPUTE, store=store,
                            store_slot=slots, accumulate=acc)
        else:
            qk_src = None
            if self._in_self_window() and K <= self.SELF_REPLACE_MAX_KEYS:
                qk_src = list(range(N))
                for n in range(n0 + 1, N):
                    qk_src[n] = n0       # P_edit <- P_source, V stays the edit's own
            _hip.self_attn(q, k, v, out, heads, scale, compute=config.COMPUTE, qk_src=qk_src, store=store,
                           store_slot=slots, accumulate=acc)
        return out


AttentionControlEdit._P2P_LIB = True


class AttentionReplace(AttentionControlEdit):
    """main.py:215-230."""

    _NATIVE = ("replace_cross_attention",)

    def replace_cross_attention(self, attn_base, att_replace):
        return torch.einsum('hpw,bwn->bhpn', attn_base, self.mapper)

    def _edit_program(self):
        return programs.replace_program(self.mapper)

    def __init__(self, prompts, num_steps: int, cross_replace_steps: float, self_replace_steps: float,
                 local_blend: Optional[LocalBlend] = None, tokenizer=None, device=None):
        super().__init__(prompts, num_steps, cross_replace_steps, self_replace_steps, local_blend,
                         tokenizer, device)
        self.mapper = seq_aligner.get_replacement_mapper(prompts, self.tokenizer).to(self.device)


AttentionReplace._P2P_LIB = True


class AttentionRefine(AttentionControlEdit):
    """main.py:233-253."""

    _NATIVE = ("replace_cross_attention",)

    def replace_cross_attention(self, attn_base, att_replace):
        gathered = attn_base[:, :, self.mapper].permute(2, 0, 1, 3)
        return gathered * self.alphas + att_replace * (1 - self.alphas)

    def _edit_program(self):
        return programs.refine_program(self.mapper, self.alphas)

    def __init__(self, prompts, num_steps: int, cross_replace_steps: float, self_replace_steps: float,
                 local_blend: Optional[LocalBlend] = None, tokenizer=None, device=None):
        super().__init__(prompts, num_steps, cross_replace_steps, self_replace_steps, local_blend,
                         tokenizer, device)
        mapper, alphas = seq_aligner.get_refinement_mapper(prompts, self.tokenizer)
        self.mapper, alphas = mapper.to(self.device), alphas.to(self.device)
        self.alphas = alphas.reshape(alphas.shape[0], 1, 1, alphas.shape[1])


AttentionRefine._P2P_LIB = True


class AttentionReweight(AttentionControlEdit):
    """main.py:256-278 (optionally chained on a Replace / Refine controller)."""

    _NATIVE = ("replace_cross_attention",)

    def replace_cross_attention(self, attn_base, att_replace):
        if self.prev_controller is not None:
            attn_base = self.prev_controller.replace_cross_attention(attn_base, att_replace)
        return attn_base[None, :, :, :] * self.equalizer[:, None, None, :]

    def _edit_program(self):
        inner = None
        prev = self.prev_controller
        if prev is not None:
            if not (isinstance(prev, AttentionControlEdit) and prev.fused_supported()):
                raise NotFusable
            inner = prev._edit_program()
            if not np.all(inner.post == 1.0):
                raise NotFusable
        return programs.reweight_program(self.equalizer, self.batch_size - 1, inner)

    def __init__(self, prompts, num_steps: int, cross_replace_steps: float, self_replace_steps: float,
                 equalizer, local_blend: Optional[LocalBlend] = None,
                 controller: Optional[AttentionControlEdit] = None, tokenizer=None, device=None):
        super().__init__(prompts, num_steps, cross_replace_steps, self_replace_steps, local_blend,
                         tokenizer, device)
        self.equalizer = equalizer.to(self.device)
        self.prev_controller = controller


AttentionReweight._P2P_LIB = True


# ============================================================================ prompt-group batching
class GroupBatch(AttentionControl):
    """Several prompt groups -- one controller each, built exactly as for a single group -- in
    ONE U-Net batch (BASELINE.json configs[2]: a batch of edit groups).  The reference runs one
    group per pipeline call (``self.batch_size = len(prompts)``, main.py:205); this build
    extension runs G of them per call: the U-Net batch is ``[uncond g0..gG-1 | cond g0..gG-1]``
    and every attention call is still ONE kernel launch, with one prompt-group descriptor per
    member (its edit program, its ``cross_replace_alpha[cur_step]`` row, its self-injection
    source, its AttentionStore slots).  Each member keeps its own counters and its own
    ``attention_store`` (views into one running-sum tensor per layer), so
    ``member.get_average_attention()``, ``aggregate_attention`` and LocalBlend work per group
    unchanged.  Members must take the fused path (library controllers, no LOW_RESOURCE)."""

    _NATIVE = ("__call__", "forward", "between_steps", "step_callback")

    def __init__(self, controllers, group_size: Optional[int] = None):
        super().__init__()
        self.members = list(controllers)
        if not self.members:
            raise ValueError("GroupBatch needs at least one controller")
        sizes = {getattr(m, "batch_size", None) for m in self.members}
        if group_size is None:
            if len(sizes) != 1 or None in sizes:
                raise ValueError("pass group_size= (members disagree on / do not know their batch size)")
            group_size = sizes.pop()
        self.group_size = int(group_size)
        for m in self.members:
            if not (isinstance(m, AttentionControl) and m.fused_supported()):
                raise ValueError(f"{type(m).__name__}: GroupBatch members must take the fused kernel path")
            # an edit controller's tables (program records, alpha rows, LocalBlend slices) are
            # sized by its own prompt count: it must equal the group size the kernels get
            if isinstance(m, AttentionControlEdit) and m.batch_size != self.group_size:
                raise ValueError(f"{type(m).__name__} was built for {m.batch_size} prompts, "
                                 f"GroupBatch groups have {self.group_size}")
        storing = {isinstance(m, AttentionStore) for m in self.members}
        if len(storing) != 1:
            raise ValueError("mix of storing and non-storing controllers")
        self._storing = storing.pop()
        if self._storing and len({bool(m.store_self_maps) for m in self.members}) != 1:
            raise ValueError("GroupBatch members disagree on store_self_maps")
        self._calls = defaultdict(int)
        self._combined = defaultdict(list)

    # counters: the composite counts like any controller and moves every member in lockstep
    @property
    def num_att_layers(self):
        return self._num_att_layers

    @num_att_layers.setter
    def num_att_layers(self, n):
        self._num_att_layers = n
        for m in getattr(self, "members", ()):
            m.num_att_layers = n

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        raise NotImplementedError("GroupBatch runs only on the fused kernels (no materialised protocol)")

    def between_steps(self):
        self._calls = defaultdict(int)

    def reset(self):
        super().reset()
        for m in getattr(self, "members", ()):
            m.reset()
        self._calls = defaultdict(int)
        self._combined = defaultdict(list)

    def step_callback(self, x_t):
        B = self.group_size
        return torch.cat([m.step_callback(x_t[g * B:(g + 1) * B]) for g, m in enumerate(self.members)])

    def fused_step_mask(self):
        fns = []
        for m in self.members:
            ok, fn = m.fused_step_mask()
            if not ok:
                return False, None
            fns.append(fn)
        if all(fn is None for fn in fns):
            return True, None
        B = self.group_size

        def mask_fn(size):
            masks = [fn(size) if fn is not None else None for fn in fns]
            if all(mk is None for mk in masks):
                return None
            folded = [mk for mk in masks if isinstance(mk, FoldedBlendMask)]
            if folded and len(folded) == sum(mk is not None for mk in masks) and \
                    len({f.latent_entry()[1:] for f in folded}) == 1:
                # every blending group folded, one threshold set: the masks are built inside
                # p2p_latent_step (one launch per step for the whole batch)
                return masks, B
            return group_mask_tensor(masks, B, size)

        return True, mask_fn

    def _fused_forward(self, q, k, v, heads, scale, is_cross, place_in_unet):
        if _low_resource():
            raise ValueError("GroupBatch does not run with LOW_RESOURCE (one U-Net call per CFG half)")
        N, P, K = q.shape[0], q.shape[1], k.shape[1]
        B, G = self.group_size, len(self.members)
        GB = G * B
        if N != 2 * GB:
            raise ValueError(f"GroupBatch of {G} x {B} prompts got a U-Net batch of {N}")
        store, acc, slots, store_key = None, False, None, None
        store_self = self._storing and all(m.store_self_maps for m in self.members)
        if self._storing and not is_cross and any(m.store_self_maps for m in self.members) and not store_self:
            raise ValueError("GroupBatch members disagree on store_self_maps")
        if self._storing and P <= MAX_STORED_QUERIES and (is_cross or store_self):
            key = f"{place_in_unet}_{'cross' if is_cross else 'self'}"
            idx = self._calls[key]
            self._calls[key] = idx + 1
            store_key = (key, idx)
            if len(self.members[0].attention_store) == 0:
                store = torch.empty(GB * heads, P, K, dtype=torch.float32, device=q.device)
                for g, m in enumerate(self.members):
                    m.step_store[key].append(store[g * B * heads:(g + 1) * B * heads])
                self._combined[key].append(store)
            else:
                store, acc = self._combined[key][idx], True
            slots = [-1] * GB + [(n - GB) * heads for n in range(GB, N)]
        out = torch.empty_like(q)
        if is_cross and K <= _hip.MAX_KEYS_CROSS:
            groups = [(0, GB, None, None, None, _hip.shared_kv_hint(k, v, 0, GB))]
            for g, m in enumerate(self.members):
                first = GB + g * B
                if isinstance(m, AttentionControlEdit):
                    alpha = m.cross_replace_alpha[m.cur_step]
                    if alpha.shape[-1] != K or alpha.device != q.device:
                        raise ValueError("edit tables do not match this attention call")
                    blend = m._blend_fold(store_key, P, K, heads, q.device) if store is not None else None
                    prog, hints = m._cross_step(q.device, K)
                    groups.append((first, B, prog, alpha.contiguous(), blend, hints))
                else:
                    groups.append((first, B, None, None))
            _hip.cross_attn(q, k, v, out, heads, scale, groups, compute=config.COMPUTE, store=store,
                            store_slot=slots, accumulate=acc)
        else:
            qk_src = list(range(N))
            for g, m in enumerate(self.members):
                if (isinstance(m, AttentionControlEdit) and not is_cross and m._in_self_window()
                        and K <= m.SELF_REPLACE_MAX_KEYS):
                    src = GB + g * B
                    for b in range(1, B):
                        qk_src[src + b] = src
            _hip.self_attn(q, k, v, out, heads, scale, compute=config.COMPUTE, qk_src=qk_src, store=store,
                           store_slot=slots, accumulate=acc)
        return out

    def attention(self, q, k, v, heads, scale, is_cross, place_in_unet, mask=None):
        if mask is not None:
            raise ValueError("GroupBatch does not take an attention mask")
        out = self._fused_forward(q, k, v, heads, scale, is_cross, place_in_unet)
        for m in self.members:
            m._advance_layer()
        self._advance_layer()
        return out


GroupBatch._P2P_LIB = True


def get_equalizer(text: str, word_select: Union[int, Tuple[int, ...]],
                  values: Union[List[float], Tuple[float, ...]], tokenizer=None):
    """main.py:281-290: one row per value, every selected word's columns set to ``values``."""
    tokenizer = tokenizer or get_tokenizer()
    if type(word_select) is int or type(word_select) is str:
        word_select = (word_select,)
    eq = torch.ones(len(values), MAX_NUM_WORDS)
    vals = torch.tensor(values, dtype=torch.float32)
    for word in word_select:
        eq[:, get_word_inds(text, word, tokenizer)] = vals
    return eq


def aggregate_attention(attention_store: AttentionStore, res: int, from_where: List[str], is_cross: bool,
                        select: int, prompts: Optional[List[str]] = None):
    """main.py:293-307 (``prompts`` is the reference's module global; defaults to the
    controller's batch size -- a plain AttentionStore has none, so pass ``prompts=`` there)."""
    n_prompts = len(prompts) if prompts is not None else getattr(attention_store, "batch_size", None)
    if n_prompts is None:
        raise ValueError(f"{type(attention_store).__name__} does not know its prompt count: pass prompts=")
    maps = attention_store.get_average_attention()
    picked = []
    for location in from_where:
        for item in maps[f"{location}_{'cross' if is_cross else 'self'}"]:
            if item.shape[1] == res ** 2:
                picked.append(item.reshape(n_prompts, -1, res, res, item.shape[-1])[select])
    out = torch.cat(picked, dim=0)
    return (out.sum(0) / out.shape[0]).cpu()


def reduce_maps(attention_store: AttentionStore, res: int, from_where: List[str], is_cross: bool,
                n_prompts: int) -> torch.Tensor:
    """aggregate_attention for every prompt at once, left on the device: the average over the
    stored layers at ``res`` and their heads of the step-averaged maps, [n_prompts, res, res, K]
    (main.py:296-307 with ``select`` = each prompt in turn; same sum order per prompt)."""
    maps = attention_store.get_average_attention()
    picked = []
    for location in from_where:
        for item in maps[f"{location}_{'cross' if is_cross else 'self'}"]:
            if item.shape[1] == res ** 2:
                picked.append(item.reshape(n_prompts, -1, res, res, item.shape[-1]))
    if not picked:
        raise ValueError(f"no stored {'cross' if is_cross else 'self'} maps at {res}x{res} in {from_where}")
    out = torch.cat(picked, dim=1)
    return out.sum(1) / out.shape[1]
