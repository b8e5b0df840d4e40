"""Oracle restatement of the controllers, LocalBlend and DDIM (torch fp32 CPU).

TEST INFRASTRUCTURE ONLY.  One class covers every reference controller through two
parameters, ``flavour`` ("main" = main.py:69-278, "null" = null_text.py:117-337) and
``kind`` (store / replace / refine / reweight).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import tables

KEYS = ("down_cross", "mid_cross", "up_cross", "down_self", "mid_self", "up_self")


class OracleController:
    def __init__(self, flavour="main", kind="store", prompts=None, num_steps=None, cross_replace_steps=None,
                 self_replace_steps=None, tok=None, equalizer=None, inner=None, local_blend=None,
                 low_resource=False, store_self=True):
        self.flavour, self.kind = flavour, kind
        self.low_resource = low_resource
        self.store_self = store_self
        self.cur_step = 0
        self.cur_att_layer = 0
        self.num_att_layers = -1
        self.step_store = {k: [] for k in KEYS}
        self.attention_store = {}
        self.local_blend = local_blend
        self.inner = inner
        if kind in ("replace", "refine", "reweight"):
            self.B = len(prompts)
            spec = dict(cross_replace_steps) if isinstance(cross_replace_steps, dict) else cross_replace_steps
            self.alpha = tables.time_word_alpha(prompts, num_steps, spec, tok)   # main.py:206
            s = self_replace_steps
            if isinstance(s, float):
                s = (0.0, s)
            self.window = (int(num_steps * s[0]), int(num_steps * s[1]))       # main.py:208-211
            self.self_max_keys = 16 ** 2 if flavour == "main" else 32 ** 2      # main.py:170 / null:225
            if kind == "replace":
                self.mapper = tables.replacement(prompts, tok)
            elif kind == "refine":
                self.mapper, a = tables.refinement(prompts, tok)
                self.ref_alphas = a.reshape(a.shape[0], 1, 1, a.shape[1])
            else:
                self.equalizer = equalizer

    # -- main.py:85-98
    def __call__(self, attn, is_cross, place):
        skip = self.num_att_layers if self.low_resource else 0
        if self.cur_att_layer >= skip:
            if self.low_resource:
                attn = self.forward(attn, is_cross, place)
            else:
                half = attn.shape[0] // 2
                attn[half:] = self.forward(attn[half:], is_cross, place)
        self.cur_att_layer += 1
        if self.cur_att_layer == self.num_att_layers + skip:
            self.cur_att_layer = 0
            self.cur_step += 1
            self.between_steps()
        return attn

    # -- main.py:129-142: store (aliasing view) then edit in place
    def forward(self, attn, is_cross, place):
        if self.kind == "empty":
            return attn
        if attn.shape[1] <= 32 ** 2 and (is_cross or self.store_self):
            self.step_store[f"{place}_{'cross' if is_cross else 'self'}"].append(attn)
        if self.kind == "store":
            return attn
        if not (is_cross or self.window[0] <= self.cur_step < self.window[1]):
            return attn
        view = attn.reshape(self.B, attn.shape[0] // self.B, *attn.shape[1:])
        base, rep = view[0], view[1:]
        if is_cross:
            a = self.alpha[self.cur_step]
            view[1:] = self.cross_edit(base, rep) * a + (1 - a) * rep
        elif rep.shape[2] <= self.self_max_keys:
            view[1:] = base.unsqueeze(0).expand(rep.shape[0], *base.shape)
        return view.reshape(self.B * view.shape[1], *attn.shape[1:])

    def cross_edit(self, base, rep):
        if self.kind == "replace":                                   # main.py:217-218
            return torch.einsum("hpw,bwn->bhpn", base, self.mapper)
        if self.kind == "refine":                                    # main.py:235-239
            g = base[:, :, self.mapper].permute(2, 0, 1, 3)
            return g * self.ref_alphas + rep * (1 - self.ref_alphas)
        if self.inner is not None:                                   # main.py:258-264
            base = self.inner.cross_edit(base, rep)
        return base[None, :, :, :] * self.equalizer[:, None, None, :]

    def between_steps(self):
        if len(self.attention_store) == 0:
            self.attention_store = self.step_store
        else:
            for k in self.attention_store:
                for i in range(len(self.attention_store[k])):
                    self.attention_store[k][i] += self.step_store[k][i]
        self.step_store = {k: [] for k in KEYS}

    def average(self):
        return {k: [t / self.cur_step for t in v] for k, v in self.attention_store.items()}

    def step_callback(self, x_t):
        if self.local_blend is not None:
            x_t = self.local_blend(x_t, self.attention_store)
        return x_t


class OracleLocalBlend:
    """main.py:35-52 (flavour "main") / null_text.py:41-70 (flavour "null")."""

    def __init__(self, flavour, prompts, words, tok, threshold=0.3, substruct_words=None, start_blend=0.2,
                 th=(0.3, 0.3), num_ddim_steps=50):
        self.flavour = flavour
        self.B = len(prompts)
        self.alpha = tables.blend_alpha(prompts, words, tok).reshape(self.B, 1, 1, 1, 1, 77)
        self.sub = None
        if substruct_words is not None:
            self.sub = tables.blend_alpha(prompts, substruct_words, tok).reshape(self.B, 1, 1, 1, 1, 77)
        self.threshold = threshold
        self.th = th
        self.start_blend = int(start_blend * num_ddim_steps)
        self.counter = 0
        self.last_mask = None

    def _mask(self, maps, alpha, pool, th, size):
        m = (maps * alpha).sum(-1).mean(1)
        if pool:
            m = F.max_pool2d(m, (3, 3), (1, 1), padding=(1, 1))
        m = F.interpolate(m, size=size)
        m = m / m.max(2, keepdim=True)[0].max(3, keepdim=True)[0]
        return m.gt(th)

    def __call__(self, x_t, store):
        maps = store["down_cross"][2:4] + store["up_cross"][:3]
        maps = torch.cat([t.reshape(self.B, -1, 1, 16, 16, 77) for t in maps], dim=1)
        size = tuple(x_t.shape[2:])
        if self.flavour == "main":
            m = self._mask(maps, self.alpha, True, self.threshold, size)
            mask = (m[:1] + m[1:]).float()
            self.last_mask = torch.cat([m[:1], m[:1] + m[1:]])
            return x_t[:1] + mask * (x_t - x_t[:1])
        self.counter += 1
        if self.counter <= self.start_blend:
            return x_t
        m = self._mask(maps, self.alpha, True, self.th[0], size)
        m = m[:1] + m
        if self.sub is not None:
            s = self._mask(maps, self.sub, False, self.th[1], size)
            m = m * ~(s[:1] + s)
        self.last_mask = m
        return x_t[:1] + m.float() * (x_t - x_t[:1])


def ddim_prev(alphas_cumprod, final_alpha, eps, t, x, n_train=1000, n_inf=50):
    """null_text.py:471-479."""
    tp = t - n_train // n_inf
    a_t = alphas_cumprod[t]
    a_p = alphas_cumprod[tp] if tp >= 0 else final_alpha
    x0 = (x - (1 - a_t) ** 0.5 * eps) / a_t ** 0.5
    return a_p ** 0.5 * x0 + (1 - a_p) ** 0.5 * eps


def ddim_next(alphas_cumprod, final_alpha, eps, t, x, n_train=1000, n_inf=50):
    """null_text.py:481-489."""
    t_cur, t_next = min(t - n_train // n_inf, 999), t
    a_t = alphas_cumprod[t_cur] if t_cur >= 0 else final_alpha
    a_n = alphas_cumprod[t_next]
    x0 = (x - (1 - a_t) ** 0.5 * eps) / a_t ** 0.5
    return a_n ** 0.5 * x0 + (1 - a_n) ** 0.5 * eps
