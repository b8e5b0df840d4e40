"""Self-attention launch time vs input layout and cache state (why the in-pipeline G2/G6 d = 80
launch is slower than the isolated A/B): q/k/v contiguous [N, P, C] or strided views of one fused
[N, P, 3C] projection output (what ptp_utils' fused QKV GEMM hands over), and the inputs hot
(one set reused) or cold (a 1 GiB buffer written between launches evicts L2 and the MALL).
Per-launch HIP events, mean of 30 launches.  Usage: python tools/layout_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402


def run(P, d, fused, cold, n=30, N=8, H=8):
    C = H * d
    if fused:
        qkv = torch.randn(N, P, 3 * C, device="cuda").to(torch.bfloat16)
        q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    else:
        q, k, v = (torch.randn(N, P, C, device="cuda").to(torch.bfloat16) for _ in range(3))
    o = torch.empty(N, P, C, device="cuda", dtype=torch.bfloat16)
    junk = torch.empty(1 << 28, device="cuda", dtype=torch.float32) if cold else None
    fn = lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5)  # noqa: E731
    for _ in range(3):
        fn()
    ev = []
    for i in range(n):
        if cold:
            junk.fill_(float(i))
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    return round(1e3 * sum(s.elapsed_time(e) for s, e in ev) / n, 2)


def main():
    out = {}
    for name, (P, d) in {"G1_d40": (4096, 40), "G2_d80": (1024, 80), "G3_d160": (256, 160)}.items():
        out[name] = {f"{'fused' if f else 'contig'}_{'cold' if c else 'hot'}_us": run(P, d, f, c)
                     for f in (False, True) for c in (False, True)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
