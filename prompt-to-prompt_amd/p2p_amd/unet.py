"""SD-v1.4-shaped U-Net with patchable ``CrossAttention`` modules (random init).

The reference runs diffusers-0.8.1's ``UNet2DConditionModel`` loaded from the SD-v1.4
checkpoint (main.py:25-30).  Neither is available offline, so this module rebuilds that
topology (block_out_channels 320/640/1280/1280, 2 layers per down block, 3 per up block,
8 heads -- diffusers-0.8.1 passes ``attention_head_dim=8`` as the head count -- cross dim
768, GEGLU feed-forward) with default-initialised weights.  What matters for the hot path is
kept exactly: 32 modules whose class is named ``CrossAttention`` with the 0.8.1 attribute
surface (``heads``, ``scale``, ``to_q/k/v``, ``to_out`` ModuleList,
``reshape_heads_to_batch_dim`` / ``reshape_batch_dim_to_heads``), called as
``attn1(x)`` then ``attn2(x, context=ctx)`` in every transformer block, in the order
down64 x2, down32 x2, down16 x2, mid8, up16 x3, up32 x3, up64 x3.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


class CrossAttention(nn.Module):
    def __init__(self, query_dim, context_dim=None, heads=8, dim_head=64, dropout=0.0):
        super().__init__()
        inner = heads * dim_head
        context_dim = context_dim if context_dim is not None else query_dim
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.to_q = nn.Linear(query_dim, inner, bias=False)
        self.to_k = nn.Linear(context_dim, inner, bias=False)
        self.to_v = nn.Linear(context_dim, inner, bias=False)
        self.to_out = nn.ModuleList([nn.Linear(inner, query_dim), nn.Dropout(dropout)])

    def reshape_heads_to_batch_dim(self, t):
        b, n, c = t.shape
        h = self.heads
        return t.reshape(b, n, h, c // h).permute(0, 2, 1, 3).reshape(b * h, n, c // h)

    def reshape_batch_dim_to_heads(self, t):
        bh, n, d = t.shape
        h = self.heads
        return t.reshape(bh // h, h, n, d).permute(0, 2, 1, 3).reshape(bh // h, n, d * h)

    def forward(self, x, context=None, mask=None):
        # unpatched: plain attention on the HIP kernels (register_attention_control replaces this)
        from .attention import plain_attention
        q = self.to_q(x)
        src = x if context is None else context
        out = plain_attention(q, self.to_k(src), self.to_v(src), self.heads, self.scale)
        return self.to_out[1](self.to_out[0](out))


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, x):
        h, gate = self.proj(x).chunk(2, dim=-1)
        return h * F.gelu(gate)


class FeedForward(nn.Module):
    def __init__(self, dim, mult=4, dropout=0.0):
        super().__init__()
        inner = dim * mult
        self.net = nn.Sequential(GEGLU(dim, inner), nn.Dropout(dropout), nn.Linear(inner, dim))

    def forward(self, x):
        return self.net(x)


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, n_heads, d_head, context_dim):
        super().__init__()
        self.attn1 = CrossAttention(dim, None, n_heads, d_head)
        self.ff = FeedForward(dim)
        self.attn2 = CrossAttention(dim, context_dim, n_heads, d_head)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.norm3 = nn.LayerNorm(dim)

    def forward(self, x, context=None):
        x = self.attn1(self.norm1(x)) + x
        x = self.attn2(self.norm2(x), context=context) + x
        return self.ff(self.norm3(x)) + x


class Transformer2DModel(nn.Module):
    def __init__(self, n_heads, d_head, in_channels, context_dim=768, groups=32):
        super().__init__()
        inner = n_heads * d_head
        self.norm = nn.GroupNorm(groups, in_channels, eps=1e-6)
        self.proj_in = nn.Conv2d(in_channels, inner, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(inner, n_heads, d_head, context_dim)])
        self.proj_out = nn.Conv2d(inner, in_channels, 1)

    def forward(self, x, encoder_hidden_states=None):
        b, c, h, w = x.shape
        res = x
        x = self.proj_in(self.norm(x))
        x = x.permute(0, 2, 3, 1).reshape(b, h * w, c)
        for blk in self.transformer_blocks:
            x = blk(x, context=encoder_hidden_states)
        x = x.reshape(b, h, w, c).permute(0, 3, 1, 2)
        return self.proj_out(x) + res


class ResnetBlock2D(nn.Module):
    def __init__(self, in_ch, out_ch, temb_ch=1280, groups=32, eps=1e-5):
        super().__init__()
        self.norm1 = nn.GroupNorm(groups, in_ch, eps=eps)
        self.conv1 = nn.Conv2d(in_ch, out_ch, 3, padding=1)
        self.time_emb_proj = nn.Linear(temb_ch, out_ch)
        self.norm2 = nn.GroupNorm(groups, out_ch, eps=eps)
        self.conv2 = nn.Conv2d(out_ch, out_ch, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(in_ch, out_ch, 1) if in_ch != out_ch else None

    def forward(self, x, temb):
        h = self.conv1(F.silu(self.norm1(x)))
        h = h + self.time_emb_proj(F.silu(temb))[:, :, None, None]
        h = self.conv2(F.silu(self.norm2(h)))
        if self.conv_shortcut is not None:
            x = self.conv_shortcut(x)
        return x + h


class Downsample2D(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, stride=2, padding=1)

    def forward(self, x):
        return self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, padding=1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class CrossAttnDownBlock2D(nn.Module):
    def __init__(self, in_ch, out_ch, layers=2, heads=8, context_dim=768, downsample=True, temb_ch=1280):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(in_ch if i == 0 else out_ch, out_ch, temb_ch)
                                      for i in range(layers)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, out_ch // heads, out_ch, context_dim)
                                         for _ in range(layers)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_ch)]) if downsample else None

    def forward(self, x, temb, ctx):
        outs = ()
        for res, att in zip(self.resnets, self.attentions):
            x = att(res(x, temb), encoder_hidden_states=ctx)
            outs += (x,)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
            outs += (x,)
        return x, outs


class DownBlock2D(nn.Module):
    def __init__(self, in_ch, out_ch, layers=2, downsample=False, temb_ch=1280):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(in_ch if i == 0 else out_ch, out_ch, temb_ch)
                                      for i in range(layers)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_ch)]) if downsample else None

    def forward(self, x, temb, ctx=None):
        outs = ()
        for res in self.resnets:
            x = res(x, temb)
            outs += (x,)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
            outs += (x,)
        return x, outs


def _up_resnets(in_ch, prev_ch, out_ch, layers, temb_ch=1280):
    mods = []
    for i in range(layers):
        skip = in_ch if i == layers - 1 else out_ch
        r_in = prev_ch if i == 0 else out_ch
        mods.append(ResnetBlock2D(r_in + skip, out_ch, temb_ch))
    return nn.ModuleList(mods)


class UpBlock2D(nn.Module):
    def __init__(self, in_ch, prev_ch, out_ch, layers=3, upsample=True, temb_ch=1280):
        super().__init__()
        self.resnets = _up_resnets(in_ch, prev_ch, out_ch, layers, temb_ch)
        self.upsamplers = nn.ModuleList([Upsample2D(out_ch)]) if upsample else None

    def forward(self, x, temb, skips, ctx=None):
        for res in self.resnets:
            x = res(torch.cat([x, skips[-1]], dim=1), temb)
            skips = skips[:-1]
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class CrossAttnUpBlock2D(nn.Module):
    def __init__(self, in_ch, prev_ch, out_ch, layers=3, heads=8, context_dim=768, upsample=True, temb_ch=1280):
        super().__init__()
        self.resnets = _up_resnets(in_ch, prev_ch, out_ch, layers, temb_ch)
        self.attentions = nn.ModuleList([Transformer2DModel(heads, out_ch // heads, out_ch, context_dim)
                                         for _ in range(layers)])
        self.upsamplers = nn.ModuleList([Upsample2D(out_ch)]) if upsample else None

    def forward(self, x, temb, skips, ctx=None):
        for res, att in zip(self.resnets, self.attentions):
            x = res(torch.cat([x, skips[-1]], dim=1), temb)
            skips = skips[:-1]
            x = att(x, encoder_hidden_states=ctx)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class UNetMidBlock2DCrossAttn(nn.Module):
    def __init__(self, ch, heads=8, context_dim=768, temb_ch=1280):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, temb_ch), ResnetBlock2D(ch, ch, temb_ch)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, ch // heads, ch, context_dim)])

    def forward(self, x, temb, ctx):
        x = self.resnets[0](x, temb)
        x = self.attentions[0](x, encoder_hidden_states=ctx)
        return self.resnets[1](x, temb)


def timestep_embedding(timesteps: torch.Tensor, dim: int, max_period: int = 10000) -> torch.Tensor:
    """Sinusoidal embedding, flip_sin_to_cos=True, downscale_freq_shift=0 (SD-v1.4)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=timesteps.device) / half
    emb = timesteps[:, None].float() * torch.exp(exponent)[None, :]
    return torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)


class TimestepEmbedding(nn.Module):
    def __init__(self, in_ch, dim):
        super().__init__()
        self.linear_1 = nn.Linear(in_ch, dim)
        self.linear_2 = nn.Linear(dim, dim)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class UNet2DConditionModel(nn.Module):
    def __init__(self, in_channels=4, out_channels=4, block_out_channels=(320, 640, 1280, 1280),
                 layers_per_block=2, heads=8, cross_attention_dim=768):
        super().__init__()
        self.in_channels = in_channels
        boc = list(block_out_channels)
        temb = boc[0] * 4
        self.conv_in = nn.Conv2d(in_channels, boc[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(boc[0], temb)
        self.down_blocks = nn.ModuleList()
        out_ch = boc[0]
        for i in range(len(boc)):
            in_ch, out_ch = out_ch, boc[i]
            last = i == len(boc) - 1
            if last:
                self.down_blocks.append(DownBlock2D(in_ch, out_ch, layers_per_block, downsample=False, temb_ch=temb))
            else:
                self.down_blocks.append(CrossAttnDownBlock2D(in_ch, out_ch, layers_per_block, heads,
                                                             cross_attention_dim, downsample=True, temb_ch=temb))
        self.mid_block = UNetMidBlock2DCrossAttn(boc[-1], heads, cross_attention_dim, temb_ch=temb)
        self.up_blocks = nn.ModuleList()
        rev = boc[::-1]
        out_ch = rev[0]
        for i in range(len(rev)):
            prev, out_ch = out_ch, rev[i]
            in_ch = rev[min(i + 1, len(rev) - 1)]
            last = i == len(rev) - 1
            if i == 0:
                self.up_blocks.append(UpBlock2D(in_ch, prev, out_ch, layers_per_block + 1, upsample=True,
                                                temb_ch=temb))
            else:
                self.up_blocks.append(CrossAttnUpBlock2D(in_ch, prev, out_ch, layers_per_block + 1, heads,
                                                         cross_attention_dim, upsample=not last, temb_ch=temb))
        self.conv_norm_out = nn.GroupNorm(32, boc[0], eps=1e-5)
        self.conv_out = nn.Conv2d(boc[0], out_channels, 3, padding=1)

    @property
    def dtype(self):
        return self.conv_in.weight.dtype

    def forward(self, sample, timestep, encoder_hidden_states):
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], dtype=torch.int64, device=sample.device)
        elif timestep.dim() == 0:
            timestep = timestep[None].to(sample.device)
        timestep = timestep.expand(sample.shape[0])
        emb = self.time_embedding(timestep_embedding(timestep, self.conv_in.out_channels).to(self.dtype))
        ctx = encoder_hidden_states.to(self.dtype)
        x = self.conv_in(sample.to(self.dtype))
        skips = (x,)
        for blk in self.down_blocks:
            x, outs = blk(x, emb, ctx)
            skips += outs
        x = self.mid_block(x, emb, ctx)
        for blk in self.up_blocks:
            n = len(blk.resnets)
            res, skips = skips[-n:], skips[:-n]
            x = blk(x, emb, res, ctx)
        x = self.conv_out(F.silu(self.conv_norm_out(x)))
        return {"sample": x}
