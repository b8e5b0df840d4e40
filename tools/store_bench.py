"""AttentionStore epilogue cost of the self kernels (main.py:129-142 default: self maps kept for
P <= 32^2): G2/G6 (P = K = 1024, d = 80) and G3 (P = K = 256, d = 160), cond half (4 entries x 8
heads) accumulated into the running sum, vs the fused kernel without a store.  Achieved HBM GB/s
counts the map read + write of the running sum (8 B per element) plus q/k/v/o.  store_us = the fused
pass (O + row lse, all N entries) + self_maps_kernel (the kept maps, cond half)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
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
    N, H, B = 8, 8, 4
    for P, d in ((1024, 80), (256, 160)):
        C = H * d
        q, k, v = (torch.randn(N, P, C, device="cuda").to(torch.bfloat16) for _ in range(3))
        o = torch.empty_like(q)
        store = torch.zeros(B * H, P, P, device="cuda")
        slots = [-1] * B + [i * H for i in range(B)]
        plain = timeit(lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5))
        stored = timeit(lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5, store=store, store_slot=slots,
                                               accumulate=True))
        bytes_ = 8.0 * B * H * P * P + 4 * N * P * C * 2
        print(json.dumps({"P": P, "d": d, "fused_us": round(plain, 1), "store_us": round(stored, 1),
                          "map_bytes_MB": round(8.0 * B * H * P * P / 1e6, 1),
                          "store_GBps": round(bytes_ / stored / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
