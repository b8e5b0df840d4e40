"""DDIM scheduler (eta = 0) with the configuration null_text.py:16-20 builds.

diffusers' DDIMScheduler is external to the reference; its deterministic step is restated
in the reference itself as ``NullInversion.prev_step`` (null_text.py:471-479) and the inverse
``next_step`` (:481-489), which this module follows (pinned by tests/golden/ddim.npz).
The beta schedule (``scaled_linear``: linspace(sqrt(b0), sqrt(b1), 1000) ** 2) and the
timestep grid (``arange(n) * (1000 // n)`` reversed, steps_offset 0) are diffusers
conventions -- parity unpinned beyond the reference's own restatement.
"""
from __future__ import annotations

import numpy as np
import torch


class _Config:
    def __init__(self, num_train_timesteps):
        self.num_train_timesteps = num_train_timesteps


class DDIMScheduler:
    def __init__(self, beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear", clip_sample=False,
                 set_alpha_to_one=False, num_train_timesteps=1000, steps_offset=0):
        if beta_schedule != "scaled_linear":
            raise NotImplementedError(beta_schedule)
        if clip_sample:
            raise NotImplementedError("clip_sample")
        self.config = _Config(num_train_timesteps)
        betas = torch.linspace(beta_start ** 0.5, beta_end ** 0.5, num_train_timesteps, dtype=torch.float32) ** 2
        self.alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
        self.final_alpha_cumprod = torch.tensor(1.0) if set_alpha_to_one else self.alphas_cumprod[0]
        self.steps_offset = steps_offset
        self.num_inference_steps = None
        self.timesteps = torch.from_numpy(np.arange(0, num_train_timesteps)[::-1].copy())

    def set_timesteps(self, num_inference_steps: int):
        self.num_inference_steps = num_inference_steps
        ratio = self.config.num_train_timesteps // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = torch.from_numpy(ts + self.steps_offset)

    def _coeffs(self, t, t_other, device):
        a_t = self.alphas_cumprod[t] if t >= 0 else self.final_alpha_cumprod
        a_o = self.alphas_cumprod[t_other] if t_other >= 0 else self.final_alpha_cumprod
        return a_t.to(device), a_o.to(device)

    def prev_step(self, model_output, timestep, sample):
        """x_{t-Δ} from x_t (null_text.py:471-479)."""
        t = int(timestep)
        prev_t = t - self.config.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self._coeffs(t, prev_t, sample.device)
        beta_t = 1 - a_t
        x0 = (sample - beta_t ** 0.5 * model_output) / a_t ** 0.5
        direction = (1 - a_prev) ** 0.5 * model_output
        return a_prev ** 0.5 * x0 + direction

    def next_step(self, model_output, timestep, sample):
        """x_{t} from x_{t-Δ} (DDIM inversion, null_text.py:481-489)."""
        t_next = int(timestep)
        t = min(t_next - self.config.num_train_timesteps // self.num_inference_steps, 999)
        a_t, a_next = self._coeffs(t, t_next, sample.device)
        beta_t = 1 - a_t
        x0 = (sample - beta_t ** 0.5 * model_output) / a_t ** 0.5
        direction = (1 - a_next) ** 0.5 * model_output
        return a_next ** 0.5 * x0 + direction

    def prev_coeffs(self, timestep):
        """The four 0-dim factors prev_step multiplies by, as host floats (for p2p_latent_step):
        (beta_t ** 0.5, a_t ** 0.5, a_prev ** 0.5, (1 - a_prev) ** 0.5), computed by the same
        f32 tensor ops as prev_step."""
        t = int(timestep)
        prev_t = t - self.config.num_train_timesteps // self.num_inference_steps
        a_t, a_prev = self._coeffs(t, prev_t, torch.device("cpu"))
        return (float((1 - a_t) ** 0.5), float(a_t ** 0.5), float(a_prev ** 0.5), float((1 - a_prev) ** 0.5))

    def next_coeffs(self, timestep):
        """The same factors for next_step (DDIM inversion)."""
        t_next = int(timestep)
        t = min(t_next - self.config.num_train_timesteps // self.num_inference_steps, 999)
        a_t, a_next = self._coeffs(t, t_next, torch.device("cpu"))
        return (float((1 - a_t) ** 0.5), float(a_t ** 0.5), float(a_next ** 0.5), float((1 - a_next) ** 0.5))

    def step(self, model_output, timestep, sample, **kw):
        return {"prev_sample": self.prev_step(model_output, timestep, sample)}
