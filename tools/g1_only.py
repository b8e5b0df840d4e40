"""Launch only the dominant kernel (G1/G7 self-attention: P = K = 4096, d = 40, N = 8, H = 8,
bf16) a fixed number of times -- the program rocprofv3 --pmc passes profile.
Usage: python tools/g1_only.py [launches] [P] [d]; P2P_SELF_VARIANT selects the kernel variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    d = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    N, H = 8, 8
    C = H * d
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
    o = torch.empty_like(q)
    for _ in range(n):
        _hip.self_attn(q, k, v, o, H, d ** -0.5)
    torch.cuda.synchronize()
    print("ok", float(o.float().abs().mean()))


if __name__ == "__main__":
    main()
