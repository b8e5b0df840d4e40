"""One cross-attention configuration launched repeatedly (for rocprofv3 PMC passes):
SD config-2 U-Net call, N = 8 (4 uncond + 4 cond), H = 8, K = 77, bf16 IO.
The uncond group's K / V rows are equal and carry SHARED_KV, edit modes the R_ONLY hint (what the
controllers pass inside cross_replace_steps).
Usage: python tools/cross_one.py [iters] [mode: plain|edit|store|edit+store] [P] [d]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip, programs, seq_aligner  # noqa: E402
from p2p_amd import pipeline as pl  # noqa: E402
from p2p_amd.tokenizer import default_tokenizer  # noqa: E402


def main(iters=20, mode="edit", P=4096, d=40):
    N, H, K, B = 8, 8, 77, 4
    mapper = seq_aligner.get_replacement_mapper(pl.north_star_prompts(), default_tokenizer())
    prog = programs.replace_program(mapper).to_device("cuda")
    alpha = torch.ones(B - 1, K, device="cuda")
    C = H * d
    g = torch.Generator(device="cuda").manual_seed(P)
    q = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
    k = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
    v = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
    # the uncond prompts "" share K / V (as in the pipeline): those rows equal, and SHARED_KV on that group
    k[1:B] = k[0]
    v[1:B] = v[0]
    o = torch.empty_like(q)
    store = torch.zeros(B * H, P, K, device="cuda") if "store" in mode else None
    slots = [-1] * B + [i * H for i in range(B)]
    # (edit modes carry the R_ONLY hint, as the controllers pass it inside cross_replace_steps)
    grp = [(0, B, None, None, None, _hip.GROUP_F_SHARED_KV), (B, B, prog if "edit" in mode else None, alpha if "edit" in mode else None, None,
                                _hip.GROUP_F_R_ONLY if "edit" in mode else 0)]
    for _ in range(iters):
        _hip.cross_attn(q, k, v, o, H, d ** -0.5, grp, store=store,
                        store_slot=slots if store is not None else None, accumulate=store is not None)
    torch.cuda.synchronize()
    print("done", mode, P, d, iters)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(int(a[0]) if a else 20, a[1] if len(a) > 1 else "edit",
         int(a[2]) if len(a) > 2 else 4096, int(a[3]) if len(a) > 3 else 40)
