"""Oracle restatement of null-text inversion (null_text.py:551-606): DDIM inversion with the
conditional U-Net, then per step Adam on the null embedding through torch autograd of the eager
patched attention (oracle.forward.install(model, None)).  TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .control import ddim_next, ddim_prev


def ddim_loop(unet, alphas_cumprod, final_alpha, timesteps, cond, latent, n_steps):
    """null_text.py:551-561: x_0 -> x_T with the conditional noise prediction."""
    out = [latent]
    latent = latent.clone().detach()
    with torch.no_grad():
        for i in range(n_steps):
            t = int(timesteps[len(timesteps) - i - 1])
            eps = unet(latent, t, encoder_hidden_states=cond)["sample"]
            latent = ddim_next(alphas_cumprod, final_alpha, eps, t, latent, n_inf=n_steps)
            out.append(latent)
    return out


def null_optimization(unet, alphas_cumprod, final_alpha, timesteps, uncond, cond, latents, n_steps, inner,
                      epsilon, guidance=7.5):
    """null_text.py:574-606."""
    embs = []
    latent_cur = latents[-1]
    for i in range(n_steps):
        uncond = uncond.clone().detach().requires_grad_(True)
        opt = torch.optim.Adam([uncond], lr=1e-2 * (1.0 - i / 100.0))
        latent_prev = latents[len(latents) - i - 2]
        t = int(timesteps[i])
        with torch.no_grad():
            eps_c = unet(latent_cur, t, encoder_hidden_states=cond)["sample"]
        for _ in range(inner):
            eps_u = unet(latent_cur, t, encoder_hidden_states=uncond)["sample"]
            eps = eps_u + guidance * (eps_c - eps_u)
            loss = F.mse_loss(ddim_prev(alphas_cumprod, final_alpha, eps, t, latent_cur, n_inf=n_steps), latent_prev)
            opt.zero_grad()
            loss.backward()
            opt.step()
            if loss.item() < epsilon + i * 2e-5:
                break
        embs.append(uncond[:1].detach())
        with torch.no_grad():
            eps = unet(torch.cat([latent_cur] * 2), t, encoder_hidden_states=torch.cat([uncond, cond]))["sample"]
            eu, ec = eps.chunk(2)
            latent_cur = ddim_prev(alphas_cumprod, final_alpha, eu + guidance * (ec - eu), t, latent_cur, n_inf=n_steps)
    return embs, latent_cur
