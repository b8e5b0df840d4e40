"""LocalBlend + latent update launch timing (HIP events, median of repeats), configs[1] shape:
B = 4 prompts, 4 x 64 x 64 latents, bf16 eps, folded word sums [4, 2, 40, 256]:
  fused     : p2p_latent_step with blend sums (latent_blend_kernel: mask + blend + CFG + DDIM)
  two_step  : p2p_localblend mask (blend_finalize_kernel) + p2p_latent_step with the mask
  plain     : p2p_latent_step without a blend
Usage: python tools/latent_bench.py [iters]   (run under rocprofv3 --kernel-trace --stats for kernel times)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip, controllers  # noqa: E402
from p2p_amd.ddim import DDIMScheduler  # noqa: E402


def timed(fn, iters):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main(iters=200):
    dev = "cuda"
    B, H, L = 4, 8, 5
    g = torch.Generator(device=dev).manual_seed(0)
    eps = torch.randn(2 * B, 4, 64, 64, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(B, 4, 64, 64, device=dev, generator=g)
    out = torch.empty_like(x)
    s = DDIMScheduler(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear", clip_sample=False,
                      set_alpha_to_one=False)
    s.set_timesteps(50)
    coeffs = s.prev_coeffs(500)
    sums = torch.rand(B, 2, L * H, 256, device=dev, generator=g)
    maps = [torch.zeros(B * H, 256, 77, device=dev) for _ in range(L)]
    alpha = torch.ones(B, 77, device=dev)
    fm = controllers.FoldedBlendMask(maps, H, alpha, None, 0.3, 0.3, (64, 64), sums)
    mask = fm.materialize()
    r = {"fused_us": timed(lambda: _hip.latent_step(eps, x, out, coeffs, 7.5, None, 0, None, [fm.latent_entry()]), iters),
         "two_step_us": timed(lambda: _hip.latent_step(eps, x, out, coeffs, 7.5, fm.materialize()), iters),
         "mask_only_us": timed(lambda: fm.materialize(), iters),
         "plain_us": timed(lambda: _hip.latent_step(eps, x, out, coeffs, 7.5, None), iters)}
    print(json.dumps({k: round(v, 2) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
