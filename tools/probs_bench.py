"""Materialise protocol cost (controllers that override forward(attn, ...), main.py:85-98):
p2p_attn_probs writes softmax(QK^T) as f32 [N*H, P, K] (ptp_utils.py:195-204), p2p_attn_pv reads
it back.  Reports us per launch and the achieved GB/s of the probability write / read."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(5):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1e3)
    return statistics.median(res)


def main():
    N, H = 8, 8
    for P, d in ((4096, 40), (1024, 80), (256, 160)):
        C = H * d
        q, k, v = (torch.randn(N, P, C, device="cuda").to(torch.bfloat16) for _ in range(3))
        o = torch.empty_like(q)
        probs = torch.empty(N * H, P, P, device="cuda")
        t_p = timeit(lambda: _hip.attn_probs(q, k, H, d ** -0.5, probs))
        os.environ["P2P_SELF_VARIANT"] = "7"
        t_nt = timeit(  # P2P_SELF_VARIANT=7: plain (temporal) stores
            lambda: _hip.attn_probs(q, k, H, d ** -0.5, probs))
        os.environ["P2P_SELF_VARIANT"] = "0"
        t_v = timeit(lambda: _hip.attn_pv(probs, v, o, H))
        nbytes = probs.numel() * 4
        print(json.dumps({"P": P, "d": d, "probs_us": round(t_p, 1), "probs_GBps": round(nbytes / t_p / 1e3, 1),
                          "probs_plain_store_us": round(t_nt, 1), "pv_us": round(t_v, 1), "pv_GBps": round(nbytes / t_v / 1e3, 1),
                          "probs_MB": round(nbytes / 1e6, 1)}), flush=True)
        del probs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
