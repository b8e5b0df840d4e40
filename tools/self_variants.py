"""A/B of the self-attention schedules (P2P_SELF_VARIANT): correctness of each variant against a
torch fp32 reference on the same bf16 inputs, then interleaved timing at the G1 shape.
Usage: python tools/self_variants.py [variants...]   (default: 4 5 6)"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402


def ref(q, k, v, H, qk_src=None):
    N, P, C = q.shape
    d = C // H
    qs = q if qk_src is None else q[qk_src]
    ks = k if qk_src is None else k[qk_src]
    qh = qs.float().reshape(N, P, H, d).permute(0, 2, 1, 3)
    kh = ks.float().reshape(N, -1, H, d).permute(0, 2, 1, 3)
    vh = v.float().reshape(N, -1, H, d).permute(0, 2, 1, 3)
    p = (qh @ kh.transpose(-1, -2) * d ** -0.5).softmax(-1)
    return (p @ vh).permute(0, 2, 1, 3).reshape(N, P, C)


def check(var, N, P, K, d, H=8, qscale=1.0, qk_src=None):
    os.environ["P2P_SELF_VARIANT"] = str(var)
    g = torch.Generator(device="cuda").manual_seed(P * 7 + K)
    C = H * d
    q = (qscale * torch.randn(N, P, C, device="cuda", generator=g)).to(torch.bfloat16)
    k = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty_like(q)
    _hip.self_attn(q, k, v, o, H, d ** -0.5, qk_src=qk_src)
    want = ref(q, k, v, H, qk_src)
    err = (o.float() - want).abs().max().item()
    return err


def main():
    variants = [int(x) for x in sys.argv[1:]] or [0, 1, 3]
    cases = [(2, 4096, 4096, 40, 1.0), (2, 4096, 4096, 40, 6.0), (2, 1000, 1000, 40, 3.0), (1, 200, 77, 40, 1.0),
             (1, 100, 33, 40, 12.0), (2, 130, 4096, 40, 2.0)]
    ok = True
    for var in variants:
        for (N, P, K, d, qs) in cases:
            err = check(var, N, P, K, d, qscale=qs)
            good = err < 2.5e-2
            ok &= good
            print(json.dumps({"variant": var, "N": N, "P": P, "K": K, "d": d, "qscale": qs, "max_abs_err": err,
                              "ok": good}), flush=True)
        err = check(var, 4, 300, 300, 40, qk_src=[0, 1, 1, 1])
        ok &= err < 2.5e-2
        print(json.dumps({"variant": var, "qk_src": True, "max_abs_err": err}), flush=True)
    if not ok:
        print("CORRECTNESS FAILED")
        sys.exit(1)
    N, H, P, d = 8, 8, 4096, 40
    C = H * d
    q = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
    k = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
    v = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
    o = torch.empty_like(q)
    fn = lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5)  # noqa: E731
    t_end = time.time() + 1.0
    while time.time() < t_end:
        fn()
    torch.cuda.synchronize()
    res = {v_: [] for v_ in variants}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(6):
        for var in variants:
            os.environ["P2P_SELF_VARIANT"] = str(var)
            fn()
            s.record()
            for _ in range(50):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[var].append(s.elapsed_time(e) / 50)
    for var in variants:
        ms = statistics.median(res[var])
        print(json.dumps({"variant": var, "median_ms": round(ms, 4), "min_ms": round(min(res[var]), 4),
                          "tflops": round(4.0 * P * P * C * N / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
