"""Time one SD-v1.4-shaped U-Net call (batch 8, 64x64 latent, bf16) in several configurations, with
every attention call on the HIP kernels (DummyController): default layout, channels_last,
MIOpen find mode (cudnn.benchmark), and a hipGraph replay of the whole call.  Also reports the host
time to enqueue one call (no sync).  Diagnostic for the caller around the hot path."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import pipeline as pl, ptp_utils  # noqa: E402


def run(channels_last, benchmark, graph, iters=20):
    torch.backends.cudnn.benchmark = benchmark
    m = pl.SyntheticStableDiffusion(device="cuda", dtype=torch.bfloat16)
    if channels_last:
        m.unet = m.unet.to(memory_format=torch.channels_last)
    ptp_utils.register_attention_control(m, None)
    x = torch.randn(8, 4, 64, 64, device="cuda")
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    ctx = torch.randn(8, 77, 768, device="cuda")
    t = torch.tensor([500], device="cuda")
    with torch.no_grad():
        for _ in range(3):
            m.unet(x, t, encoder_hidden_states=ctx)
        torch.cuda.synchronize()
        fn = lambda: m.unet(x, t, encoder_hidden_states=ctx)  # noqa: E731
        if graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    m.unet(x, t, encoder_hidden_states=ctx)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                m.unet(x, t, encoder_hidden_states=ctx)
            fn = g.replay
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3, enq * 1e3


if __name__ == "__main__":
    configs = ((False, False, False), (True, False, False), (True, True, False), (False, True, False),
               (True, True, True), (False, False, True))
    if "--quick" in sys.argv:
        configs = configs[:1]
    for cl, bm, gr in configs:
        ms, enq = run(cl, bm, gr)
        print(f"[P2P_FUSE_QKV={os.environ.get('P2P_FUSE_QKV', '1')}] unet bf16 channels_last={cl} benchmark={bm} graph={gr}: {ms:.2f} ms/call (enqueue {enq:.2f} ms)",
              flush=True)
