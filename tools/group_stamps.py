"""Where the group-coupled cross kernel's time goes (experiments build, P2P_SELF_VARIANT=123: clock
stamps of wave 0..3 at the phase boundaries of cross_group_kernel, p2p_cross.hip).  Config-2 G1
launch (N = 8 = 4 uncond + 4 cond, H = 8, P = 4096, d = 40, K = 77, bf16, AttentionReplace on the
cond group), optionally G2 with stores.  Per-phase medians (cycles) for the uncond and the edit
groups, per entry.
Usage: P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=123 python tools/group_stamps.py"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from p2p_amd import _hip, programs, seq_aligner  # noqa: E402
from p2p_amd import pipeline as pl  # noqa: E402
from p2p_amd.tokenizer import default_tokenizer  # noqa: E402

NWG, W, SLOTS = 2048, 4, 24


def group_of(logical, nq, H, G):
    """cross_group_kernel's group index of a logical workgroup id (p2p_cross.hip work order: blocks
    of 4 query tiles; heads, then tiles, then groups alternating last / first)."""
    nfb, per_full = nq // 4, 4 * H * G
    if logical < nfb * per_full:
        rest = (logical % per_full) // H // 4
    else:
        r = nq - nfb * 4
        rest = ((logical - nfb * per_full) // H) // r
    return G - 1 - rest // 2 if rest % 2 == 0 else rest // 2


def run(name, P, d, store):
    N, H, K, B = 8, 8, 77, 4
    C = H * d
    tok = default_tokenizer()
    mapper = seq_aligner.get_replacement_mapper(pl.north_star_prompts(), tok)
    prog = programs.replace_program(mapper).to_device("cuda")
    alpha = torch.ones(B - 1, K, device="cuda")
    q = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
    k = torch.randn(N, K, C, device="cuda").to(torch.bfloat16)
    v = torch.randn(N, K, C, device="cuda").to(torch.bfloat16)
    k[1:B] = k[0]      # the uncond prompts "" share K / V (SHARED_KV), as in the pipeline
    v[1:B] = v[0]
    o = torch.empty_like(q)
    st = torch.zeros(B * H, P, K, device="cuda") if store else None
    slots = [-1] * B + [i * H for i in range(B)] if store else None
    grp = [(0, B, None, None, None, int(os.environ.get("STAMPS_SHARED_KV", "1")) * _hip.GROUP_F_SHARED_KV),
           (B, B, prog, alpha, None, _hip.GROUP_F_R_ONLY)]   # (alpha 1: the hint)
    fn = _hip.lib().p2p_diag_group_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    for _ in range(10):
        _hip.cross_attn(q, k, v, o, H, d ** -0.5, grp, store=st, store_slot=slots, accumulate=store)
    torch.cuda.synchronize()
    assert fn(None, 0) == 0
    _hip.cross_attn(q, k, v, o, H, d ** -0.5, grp, store=st, store_slot=slots, accumulate=store)
    torch.cuda.synchronize()
    buf = np.zeros(NWG * W * SLOTS, dtype=np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    s = buf.reshape(NWG, W, SLOTS).astype(np.int64)
    nq = (P + 127) // 128
    nwg = min(NWG, nq * H * 2)
    s = s[:nwg]
    gi = np.array([group_of(i, nq, H, 2) for i in range(nwg)])   # the kernel's work order
    print(f"== {name}: P={P} d={d} store={store}: {nwg} workgroups")
    for label, sel in (("edit group", gi == 1), ("uncond group", gi == 0)):
        ss = s[sel]
        t0 = ss[:, :, 0]
        parts = [f"prologue {np.median(ss[:, :, 1] - t0):.0f}"]
        for b in range(B):
            base = 2 + 5 * b
            prev = ss[:, :, 1] if b == 0 else ss[:, :, base - 1]
            parts.append(f"e{b}: qk+soft {np.median(ss[:, :, base] - prev):.0f} R+blend "
                         f"{np.median(ss[:, :, base + 1] - ss[:, :, base]):.0f} store "
                         f"{np.median(ss[:, :, base + 2] - ss[:, :, base + 1]):.0f} pv+O "
                         f"{np.median(ss[:, :, base + 3] - ss[:, :, base + 2]):.0f} sync+next "
                         f"{np.median(ss[:, :, base + 4] - ss[:, :, base + 3]):.0f}")
        if B > 2:   # entry 1's sync+next split: first barrier | write_entry (vmcnt(0) + LDS writes) | barrier + flags
            parts.append(f"e1 sync+next = barrier {np.median(ss[:, :, 22] - ss[:, :, 10]):.0f} | wait + LDS writes "
                         f"{np.median(ss[:, :, 23] - ss[:, :, 22]):.0f} | barrier + flags "
                         f"{np.median(ss[:, :, 11] - ss[:, :, 23]):.0f}")
        total = np.median(ss[:, :, 2 + 5 * (B - 1) + 4] - t0)
        print(f"  {label} ({len(ss)} wg): total {total:.0f}\n    " + "\n    ".join(parts))
    starts = np.sort(s[:, 0, 0] - s[:, 0, 0].min())
    ends = s[:, :, 2 + 5 * (B - 1) + 4].max(1)
    print(f"  span {ends.max() - s[:, 0, 0].min()} cycles; start median {np.median(starts):.0f}, "
          f"p90 {np.percentile(starts, 90):.0f}, last {starts[-1]}")


if __name__ == "__main__":
    run("G1", 4096, 40, False)
