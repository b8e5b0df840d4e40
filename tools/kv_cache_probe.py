"""What the cross-attention K/V projection cache (ptp_utils._cross_kv) saves per U-Net call:
(1) the 16 cross K/V GEMMs it removes, each timed alone with HIP events on the configs[1] context
([8, 77, 768] bf16 -> [8, 77, 2C]); (2) one configs[1]-shaped U-Net call (batch 8, 64x64 latent, plain
attention on the HIP kernels) with the cache on and off, alternated, median of the rounds.
Usage: python tools/kv_cache_probe.py [rounds]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from p2p_amd import pipeline as pl  # noqa: E402
from p2p_amd import ptp_utils as pu  # noqa: E402


def timed(fn, n=20):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def main(rounds=7):
    model = pl.SyntheticStableDiffusion(device="cuda", dtype=torch.bfloat16)
    prompts = pl.north_star_prompts()
    pu.register_attention_control(model, None)   # plain attention on the HIP kernels (no controller state)
    ids = model.tokenizer(prompts, padding="max_length", max_length=77, return_tensors="pt").input_ids.cuda()
    uids = model.tokenizer([""] * 4, padding="max_length", max_length=77, return_tensors="pt").input_ids.cuda()
    ctx = pu.unet_context(model, torch.cat([model.text_encoder(uids)[0], model.text_encoder(ids)[0]]))
    gemm_ms = 0.0
    n_mod = 0
    with torch.no_grad():
        for m in model.unet.modules():
            if type(m).__name__ == "CrossAttention" and m.to_k.in_features == ctx.shape[-1]:
                w = pu._stacked_weight(m, ("to_k", "to_v"))
                gemm_ms += timed(lambda: torch.nn.functional.linear(ctx, w))
                n_mod += 1
        print(f"{n_mod} cross K/V GEMMs ([8, 77, 768] x [768, 2C], bf16): {gemm_ms * 1e3:.1f} us per U-Net call "
              f"when timed alone", flush=True)
        x = torch.randn(8, 4, 64, 64, device="cuda")
        t = torch.tensor([500], device="cuda")

        def call():
            model.unet(x, t, encoder_hidden_states=ctx)
        res = {True: [], False: []}
        for _ in range(rounds):
            for cache in (False, True):
                pu.CACHE_CROSS_KV = cache
                res[cache].append(timed(call, 10))
        pu.CACHE_CROSS_KV = True
    off, on = statistics.median(res[False]), statistics.median(res[True])
    print(f"U-Net call (batch 8, 64x64, plain HIP attention): cache off {off:.3f} ms, on {on:.3f} ms "
          f"(median of {rounds} alternated rounds of 10 calls): {1e3 * (off - on):.1f} us per call")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 7)
