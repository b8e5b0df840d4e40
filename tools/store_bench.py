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
    """The running sums rotate over enough buffers (>= 1 GiB) that none stays in the 256 MB
    Infinity Cache between its launches -- as in the pipeline, where five G2/G6 layers keep 670 MB
    of self maps.  P2P_SELF_VARIANT=6 times the maps kernel with plain (temporal) accesses."""
    N, H, B = 8, 8, 4
    for P, d in ((1024, 80), (256, 160)):
        C = H * d
        q, k, v = (torch.randn(N, P, C, device="cuda").to(torch.bfloat16) for _ in range(3))
        o = torch.empty_like(q)
        map_bytes = 4 * B * H * P * P
        nbuf = max(2, -(-(1 << 30) // map_bytes))
        stores = [torch.zeros(B * H, P, P, device="cuda") for _ in range(nbuf)]
        slots = [-1] * B + [i * H for i in range(B)]
        it = [0]

        def stored():
            st = stores[it[0] % nbuf]
            it[0] += 1
            _hip.self_attn(q, k, v, o, H, d ** -0.5, store=st, store_slot=slots, accumulate=True)

        plain = timeit(lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5))
        res = {"P": P, "d": d, "fused_us": round(plain, 1), "map_bytes_MB": round(2 * map_bytes / 1e6, 1),
               "rotating_buffers": nbuf}
        for name, var in (("store_us", "0"), ("store_us_plain_access", "6")):
            os.environ["P2P_SELF_VARIANT"] = var
            t = timeit(stored, iters=4 * nbuf)
            res[name] = round(t, 1)
            res[name.replace("_us", "_GBps")] = round((2.0 * map_bytes + 4 * N * P * C * 2) / t / 1e3, 1)
        os.environ["P2P_SELF_VARIANT"] = "0"
        print(json.dumps(res), flush=True)
        del stores
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
