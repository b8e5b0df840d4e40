"""Per-geometry timing of the fused attention kernels (HIP events on the launch stream) for the
SD-v1.4 config-2 U-Net call (N = 8, H = 8).  Reports algorithmic TFLOP/s (4*P*K*C*N, unpadded)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402

GEOMS = [("G1 self", 4096, 4096, 40), ("G2 self", 1024, 1024, 80), ("G3 self", 256, 256, 160),
         ("G4 self", 64, 64, 160), ("G1 cross", 4096, 77, 40), ("G2 cross", 1024, 77, 80),
         ("G3 cross", 256, 77, 160)]


def time_fn(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main(dtype=torch.bfloat16, compute="bf16"):
    N, H = 8, 8
    out = []
    for name, P, K, d in GEOMS:
        C = H * d
        q = torch.randn(N, P, C, device="cuda").to(dtype)
        k = torch.randn(N, K, C, device="cuda").to(dtype)
        v = torch.randn(N, K, C, device="cuda").to(dtype)
        o = torch.empty_like(q)
        if "cross" in name:
            groups = [(n, 1, None, None) for n in range(N)]
            fn = lambda: _hip.cross_attn(q, k, v, o, H, d ** -0.5, groups, compute=compute)  # noqa: E731
        else:
            fn = lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5, compute=compute)  # noqa: E731
        ms = time_fn(fn)
        flop = 4.0 * P * K * C * N
        r = {"geom": name, "P": P, "K": K, "d": d, "ms": round(ms, 4), "tflops": round(flop / ms / 1e9, 1)}
        print(json.dumps(r), flush=True)
        out.append(r)
    return out


if __name__ == "__main__":
    main()
    # tile-shape variants of the fused self kernel: in-process A/B, 1 s of warm-up at load,
    # 6 interleaved rounds of 100 launches each, median per variant
    import statistics
    N, H = 8, 8
    for P, d in ((4096, 40), (1024, 80)):
        C = H * d
        q = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
        k = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
        v = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
        o = torch.empty_like(q)
        fn = lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5)  # noqa: E731
        import time as _t
        t_end = _t.time() + 1.0
        while _t.time() < t_end:
            fn()
        torch.cuda.synchronize()
        res = {var: [] for var in range(4)}
        for rnd in range(6):
            for var in range(4):
                os.environ["P2P_SELF_VARIANT"] = str(var)
                res[var].append(time_fn(fn, iters=100, warm=3))
        for var in range(4):
            ms = statistics.median(res[var])
            print(json.dumps({"variant": var, "P": P, "d": d, "median_ms": round(ms, 4), "min_ms": round(min(res[var]), 4),
                              "tflops_median": round(4.0 * P * P * C * N / ms / 1e9, 1)}), flush=True)
        os.environ["P2P_SELF_VARIANT"] = "0"
