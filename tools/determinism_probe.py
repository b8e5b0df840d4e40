"""Run-to-run reproducibility of the pieces of one edit group (diagnostic): the same inputs twice
through (1) the hot-path kernels alone (self / cross attention at the G1..G4 shapes, with a Replace
program and stores), (2) one U-Net call with every attention on the HIP kernels, (3) one U-Net call
with the unpatched forward (plain HIP attention), (4) the U-Net's GEMMs (nn.Linear at the U-Net's shapes) and
convolutions alone.  Prints whether each pair is bit-identical and the max |diff|."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from p2p_amd import _hip, controllers, ptp_utils  # noqa: E402
from p2p_amd import pipeline as pl  # noqa: E402


def same(label, a, b):
    eq = torch.equal(a, b)
    print(f"{label:60s} equal {eq}  max|diff| {(a.float() - b.float()).abs().max().item():.3e}", flush=True)
    return eq


def kernels():
    g = torch.Generator(device="cuda").manual_seed(0)
    for P, K, d in ((4096, 4096, 40), (1024, 1024, 80), (256, 256, 160), (64, 64, 160)):
        C = 8 * d
        q, k, v = (torch.randn(8, n, C, device="cuda", generator=g).bfloat16() for n in (P, K, K))
        outs = []
        for _ in range(2):
            o = torch.empty_like(q)
            _hip.self_attn(q, k, v, o, 8, d ** -0.5)
            outs.append(o)
        same(f"self attention P={P} d={d}", *outs)
        kc, vc = (torch.randn(8, 77, C, device="cuda", generator=g).bfloat16() for _ in range(2))
        outs = []
        for _ in range(2):
            o = torch.empty_like(q)
            _hip.cross_attn(q, kc, vc, o, 8, d ** -0.5, [(0, 8, None, None)])
            outs.append(o)
        same(f"cross attention (plain) P={P} d={d}", *outs)


def unet(attn):
    m = pl.SyntheticStableDiffusion(device="cuda", dtype=torch.bfloat16)
    if attn == "hip":
        ptp_utils.register_attention_control(m, controllers.EmptyControl())
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(8, 4, 64, 64, device="cuda", generator=g)
    ctx = torch.randn(8, 77, 768, device="cuda", generator=g).bfloat16()
    t = torch.tensor([500], device="cuda")
    with torch.no_grad():
        m.unet(x, t, encoder_hidden_states=ctx)
        a = m.unet(x, t, encoder_hidden_states=ctx)["sample"].clone()
        b = m.unet(x, t, encoder_hidden_states=ctx)["sample"].clone()
    same(f"U-Net call, attention on {attn}", a, b)
    return m


def layers(m):
    g = torch.Generator(device="cuda").manual_seed(2)
    with torch.no_grad():
        for name, mod in m.unet.named_modules():
            if isinstance(mod, torch.nn.Linear) and name.endswith(("ff.net.2", "to_q", "proj_in")):
                x = torch.randn(8, 4096 if "down_blocks.0" in name or "up_blocks.3" in name else 256, mod.in_features,
                                device="cuda", generator=g).bfloat16()
                same(f"linear {name} {tuple(x.shape)} -> {mod.out_features}", mod(x), mod(x))
            if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size == (3, 3) and name.endswith("conv1"):
                hw = 64 if "blocks.0" in name else 32
                x = torch.randn(16, mod.in_channels, hw, hw, device="cuda", generator=g).bfloat16()
                same(f"conv {name} {tuple(x.shape)}", mod(x), mod(x))


if __name__ == "__main__":
    kernels()
    unet("unpatched")
    layers(unet("hip"))
    torch.backends.cudnn.deterministic = True
    print("torch.backends.cudnn.deterministic = True")
    unet("hip")
