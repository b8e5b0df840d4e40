"""Self-attention launch timing at the small SD geometries (config-2 U-Net call: N = 8, H = 8,
bf16 IO, O only): G2 (P = K = 1024, d = 80), G3 (256, 160), G4 (64, 160).  GPU time per launch
from captured HIP graphs (no host enqueue), median of 5 replays x 50 launches.
Usage: [P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=v] python tools/small_bench.py"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402
from cross_bench import time_graph  # noqa: E402


def main():
    out = {"variant": int(os.environ.get("P2P_SELF_VARIANT", "0"))}
    for name, P, d in (("G2", 1024, 80), ("G3", 256, 160), ("G4", 64, 160)):
        N, H = 8, 8
        C = H * d
        g = torch.Generator(device="cuda").manual_seed(P)
        q = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
        k = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
        v = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
        o = torch.empty_like(q)
        fn = lambda: _hip.self_attn(q, k, v, o, H, d ** -0.5)  # noqa: E731
        us = statistics.median(time_graph(fn, 50) for _ in range(5))
        flop = 4.0 * P * P * C * N
        out[name + "_us"] = round(us, 2)
        out[name + "_frac"] = round(flop / (us * 1e-6) / 2.5e15, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
