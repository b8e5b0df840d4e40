"""Oracle restatement of the patched CrossAttention.forward (ptp_utils.py:183-208) and of the
hook that installs it (ptp_utils.py:223-242).  fp32 torch on CPU.  TEST INFRASTRUCTURE ONLY.
"""
from __future__ import annotations

import torch


def eager_attention(module, x, context, controller, place):
    """q/k/v projections, head split, QK^T*scale, softmax, controller, PV, merge, to_out."""
    b, n, _ = x.shape
    H = module.heads
    q = module.to_q(x)
    is_cross = context is not None
    src = context if is_cross else x
    k = module.to_k(src)
    v = module.to_v(src)

    def split(t):
        # the attention math always runs in fp32 (the reference's model dtype, main.py:29): a bf16
        # U-Net's projections are upcast here and the result cast back before to_out
        t = t.float()
        return t.reshape(b, t.shape[1], H, t.shape[2] // H).permute(0, 2, 1, 3).reshape(b * H, t.shape[1], -1)

    q, k, v = split(q), split(k), split(v)
    attn = (torch.einsum("bid,bjd->bij", q, k) * module.scale).softmax(dim=-1)
    if controller is not None:
        attn = controller(attn, is_cross, place)
    out = torch.einsum("bij,bjd->bid", attn, v)
    out = out.reshape(b, H, n, -1).permute(0, 2, 1, 3).reshape(b, n, -1).to(x.dtype)
    to_out = module.to_out[0] if isinstance(module.to_out, torch.nn.ModuleList) else module.to_out
    return to_out(out)


def install(model, controller):
    """Patch every CrossAttention under unet.{down,mid,up}* with the eager forward."""

    def patch(net, place):
        if net.__class__.__name__ == "CrossAttention":
            def fwd(x, context=None, mask=None, encoder_hidden_states=None, attention_mask=None, _m=net):
                return eager_attention(_m, x, context, controller, place)
            net.forward = fwd
            return 1
        return sum(patch(c, place) for c in net.children())

    count = 0
    for name, net in model.unet.named_children():
        for place in ("down", "up", "mid"):
            if place in name:
                count += patch(net, place)
                break
    if controller is not None:
        controller.num_att_layers = count
    return count
