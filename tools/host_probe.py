"""Is the U-Net call host-bound?  Host time to enqueue one configs[1]-shaped U-Net call (batch 8,
64x64 latent, bf16, every attention call on the HIP kernels) against its GPU time (a hipGraph
replay of the same call), with torch's sync-debug mode reporting any synchronising torch op.
Then the same for one edit-group denoising step of the bench pipeline (run_edit_groups, 4 steps).
Usage: python tools/host_probe.py"""
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from p2p_amd import pipeline as pl, ptp_utils  # noqa: E402


def main():
    m = pl.SyntheticStableDiffusion(device="cuda", dtype=torch.bfloat16)
    ptp_utils.register_attention_control(m, None)
    x = torch.randn(8, 4, 64, 64, device="cuda")
    ctx = torch.randn(8, 77, 768, device="cuda", dtype=torch.bfloat16)
    t = torch.tensor([500], device="cuda")
    with torch.no_grad():
        for _ in range(3):
            m.unet(x, t, encoder_hidden_states=ctx)
        torch.cuda.synchronize()
        torch.cuda.set_sync_debug_mode("warn")
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            m.unet(x, t, encoder_hidden_states=ctx)
        torch.cuda.set_sync_debug_mode(0)
        syncs = [str(x.message)[:160] for x in w if "synchroniz" in str(x.message)]
        print(f"synchronising torch ops in one U-Net call: {len(syncs)}", flush=True)
        for s in syncs[:10]:
            print("  ", s)
        torch.cuda.synchronize()
        # host enqueue of 5 calls back to back, then the GPU's drain
        t0 = time.perf_counter()
        for _ in range(5):
            m.unet(x, t, encoder_hidden_states=ctx)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"5 U-Net calls: host enqueue {1e3 * (t1 - t0) / 5:.2f} ms/call, wall {1e3 * (t2 - t0) / 5:.2f} ms/call",
              flush=True)
        # host-only: the Python / dispatch cost with the GPU idle-free (the per-op launch work)
        import torch.autograd.profiler as prof  # noqa: F401
        t0 = time.perf_counter()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as p:
            m.unet(x, t, encoder_hidden_states=ctx)
        torch.cuda.synchronize()
        print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=25), flush=True)


if __name__ == "__main__":
    main()
