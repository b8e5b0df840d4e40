"""Where the cross-attention kernel's time goes (experiments build, P2P_SELF_VARIANT=90: clock
stamps per wave at the phase boundaries of cross_attn_kernel).  Config-2 launches (N = 8, H = 8,
K = 77, bf16) at G1 (P = 4096, d = 40, AttentionReplace edit) and G3 (P = 256, d = 160, edit + map
store + LocalBlend word sums).  Prints per-phase medians (cycles) for plain and edit entries and
the launch's span (first start to last end).
Usage: P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=90 python tools/cross_stamps.py"""
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

NWG, W, SLOTS = 4096, 4, 24
PLAIN = [(0, 1, "loads issued"), (1, 2, "LDS staged + barrier"), (2, 3, "QK + softmax"), (3, 4, "PV"),
         (4, 5, "O store")]
EDIT = [(0, 19, "  (dense) loads issued"), (19, 20, "  (dense) mapper landed"), (20, 21, "  (dense) coeffs"),
        (21, 22, "  (dense) K_src landed"), (22, 8, "  (dense) barrier"), (0, 8, "src stage + barrier"), (0, 11, "start -> own softmax"), (8, 9, "P0"), (9, 10, "R = P0 M + barrier"), (10, 11, "own stage + barrier"),
        (11, 12, "own QK + softmax"), (12, 13, "blend"), (13, 14, "store epilogue"), (14, 15, "PV"),
        (13, 16, "  store: sync + slab write"), (16, 17, "  store: sync"), (17, 18, "  store: blend sums"),
        (18, 14, "  store: read-add-write")]


def run(name, P, d, store, blend, hint=0):
    N, H, K, B = 8, 8, 77, 4
    C = H * d
    tok = default_tokenizer()
    mapper = seq_aligner.get_replacement_mapper(pl.north_star_prompts(), tok)
    prog = programs.replace_program(mapper).to_device("cuda")
    alpha = torch.ones(B - 1, K, device="cuda")
    q = torch.randn(N, P, C, device="cuda").to(torch.bfloat16)
    k = torch.randn(N, K, C, device="cuda").to(torch.bfloat16)
    v = torch.randn(N, K, C, device="cuda").to(torch.bfloat16)
    o = torch.empty_like(q)
    st = torch.zeros(B * H, P, K, device="cuda") if store else None
    slots = [-1] * B + [i * H for i in range(B)] if store else None
    grp = [(0, B, None, None), (B, B, prog, alpha, None, hint)]
    if blend:
        grp[1] = (B, B, prog, alpha, (torch.zeros(B, 2, 5 * H, P, device="cuda"), torch.rand(B, K, device="cuda"),
                                      None, 0, 5 * H), hint)
    fn = _hip.lib().p2p_diag_cross_stamps
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
    nwg = nq * H * N
    s = s[:nwg]
    # the kernel's work order: entries fastest (rotated by N/2 in the second 32 of every 64 ids
    # when N divides 32), then heads, then query tiles
    ids = np.arange(nwg)
    rot = ((ids >> 5) & 1) * (N // 2) if 32 % N == 0 else 0
    ent = N - 1 - (ids % N + rot) % N
    t0 = s[:, :, 0]
    print(f"== {name}: P={P} d={d} store={store} blend={blend}: {nwg} workgroups")
    plain = ent < B + 1 if not store else ent < B
    src = (ent == B) & ~plain
    edit = ent > B
    for label, sel, phases in (("plain", plain, PLAIN), ("source", src, EDIT), ("edit", edit, EDIT)):
        ss = s[sel]
        if not len(ss):
            continue
        end = ss[:, :, 5] if label == "plain" else ss[:, :, 15]
        parts = [f"{lab} {np.median(ss[:, :, b] - ss[:, :, a]):.0f}" for a, b, lab in phases
                 if (ss[:, :, b] > 0).all() and (ss[:, :, a] > 0).all()]
        print(f"  {label:5s} ({len(ss)} wg): total {np.median(end - ss[:, :, 0]):.0f} | " + ", ".join(parts))
    ends = np.where(s[:, :, 15] > 0, s[:, :, 15], s[:, :, 5])
    span = ends.max() - t0.min()
    starts = np.sort(t0[:, 0] - t0.min())
    print(f"  launch span {span} cycles; workgroup start times: median {np.median(starts):.0f}, "
          f"p90 {np.percentile(starts, 90):.0f}, last {starts[-1]}")


if __name__ == "__main__":
    run("G2", 1024, 80, True, False)
    run("G2 R_ONLY", 1024, 80, True, False, _hip.GROUP_F_R_ONLY)
    run("G3", 256, 160, True, True)
    run("G3 R_ONLY", 256, 160, True, True, _hip.GROUP_F_R_ONLY)
    run("G4 R_ONLY", 64, 160, True, False, _hip.GROUP_F_R_ONLY)
