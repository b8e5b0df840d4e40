"""Time one SD-v1.4-shaped U-Net call (batch 8, 64x64 latent) in several layouts/dtypes, with every
attention call on the HIP kernels (DummyController).  Diagnostic for the caller around the hot path."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import pipeline as pl, ptp_utils  # noqa: E402


def run(dtype, channels_last, iters=10):
    m = pl.SyntheticStableDiffusion(device="cuda", dtype=dtype)
    if channels_last:
        m.unet = m.unet.to(memory_format=torch.channels_last)
    ptp_utils.register_attention_control(m, None)
    x = torch.randn(8, 4, 64, 64, device="cuda")
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    ctx = torch.randn(8, 77, 768, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            m.unet(x, torch.tensor(500), encoder_hidden_states=ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            m.unet(x, torch.tensor(500), encoder_hidden_states=ctx)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


if __name__ == "__main__":
    for dtype in (torch.bfloat16,):
        for cl in (False, True):
            print(f"unet {dtype} channels_last={cl}: {run(dtype, cl):.2f} ms/call", flush=True)
