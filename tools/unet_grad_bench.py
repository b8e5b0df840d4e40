"""Is the null-text inner step (batch-1 U-Net forward + backward to the null embedding, bf16)
GPU- or launch-bound?  Times N iterations end to end and the host time to enqueue them."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import pipeline as pl, ptp_utils  # noqa: E402


def main(iters=20):
    m = pl.SyntheticStableDiffusion(device="cuda", dtype=torch.bfloat16)
    ptp_utils.register_attention_control(m, None)
    x = torch.randn(1, 4, 64, 64, device="cuda")
    t = torch.tensor([500], device="cuda")
    emb = torch.randn(1, 77, 768, device="cuda", requires_grad=True)

    def step():
        eps = m.unet(x, t, encoder_hidden_states=emb)["sample"]
        loss = eps.float().square().mean()
        loss.backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"batch-1 fwd+bwd: {1e3 * t_all / iters:.2f} ms/iter wall, host enqueue {1e3 * t_enq / iters:.2f} ms/iter")
    with torch.no_grad():
        for _ in range(3):
            m.unet(x, t, encoder_hidden_states=emb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            m.unet(x, t, encoder_hidden_states=emb)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
    print(f"batch-1 fwd only: {1e3 * t_all / iters:.2f} ms/iter wall, host enqueue {1e3 * t_enq / iters:.2f} ms/iter")


if __name__ == "__main__":
    main()
