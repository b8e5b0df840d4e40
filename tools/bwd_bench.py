"""Attention backward timing (p2p_attn_bwd: delta, dQ pass, dK/dV pass + split reduction) at the null-text geometries
(U-Net batch 1: self G1 P=K=4096 d=40, G2 P=K=1024 d=80, G3 P=K=256 d=160, cross G1 K=77), HIP events,
kernel times from rocprofv3 --kernel-trace --stats (the HIP-event numbers include launch overhead)."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402

GEOMS = [("G1 self", 4096, 4096, 40), ("G2 self", 1024, 1024, 80), ("G3 self", 256, 256, 160),
         ("G1 cross", 4096, 77, 40), ("G2 cross", 1024, 77, 80)]


def main(variants):
    N, H = 1, 8
    for name, P, K, d in GEOMS:
        C = H * d
        g = torch.Generator(device="cuda").manual_seed(P + K)
        q = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
        k = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
        v = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
        dout = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
        o = torch.empty_like(q)
        lse = torch.empty(N * H, P, device="cuda")
        _hip.attn_fwd_lse(q, k, v, o, H, d ** -0.5, lse)
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
        delta = torch.empty(N * H, P, device="cuda")

        def fn():
            _hip.attn_bwd(q, k, v, o, dout, lse, H, d ** -0.5, dq, dk, dv, delta)

        ref = None
        for var in variants:
            os.environ["P2P_BWD_VARIANT"] = str(var)
            fn()
            torch.cuda.synchronize()
            cur = (dq.float().clone(), dk.float().clone(), dv.float().clone())
            if ref is None:
                ref = cur
            else:
                for a_, b_ in zip(ref, cur):
                    assert torch.allclose(a_, b_, atol=1e-2 * b_.abs().max().item()), (name, var)
        res = {x: [] for x in variants}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            for var in variants:
                os.environ["P2P_BWD_VARIANT"] = str(var)
                fn()
                s.record()
                for _ in range(20):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res[var].append(s.elapsed_time(e) / 20 * 1e3)
        flop = 2.5 * 4.0 * P * K * C * N
        for var in variants:
            med = statistics.median(res[var])
            print(json.dumps({"geom": name, "variant": var, "median_us": round(med, 1),
                              "tflops": round(flop / med / 1e6, 1)}), flush=True)
    os.environ["P2P_BWD_VARIANT"] = "0"


if __name__ == "__main__":
    main([int(x) for x in sys.argv[1:]] or [0])
