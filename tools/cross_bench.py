"""Cross-attention kernel timing by cost component (HIP events on the launch stream), SD-v1.4
config-2 U-Net call (N = 8 = 4 uncond + 4 cond, H = 8, K = 77, bf16 IO):
  plain       : no edit program, no store
  edit        : north-star AttentionReplace program on the cond group
  store       : no edit, cond-half maps accumulated into the store
  edit+store  : both (what G2/G3/G5/G6 run every step)
Usage: [CROSS_BENCH_GRAPH=1] python tools/cross_bench.py [iters]   (graph mode: GPU time without the
host enqueue, which otherwise floors every launch at ~11 us)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import torch  # noqa: E402

from p2p_amd import _hip, programs, seq_aligner  # noqa: E402
from p2p_amd import pipeline as pl  # noqa: E402
from p2p_amd.tokenizer import default_tokenizer  # noqa: E402

GEOMS = [("G1", 4096, 40), ("G2", 1024, 80), ("G3", 256, 160), ("G4", 64, 160)]


def time_fn(fn, iters, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def time_graph(fn, iters, reps=5):
    """GPU time per launch without the Python + ctypes enqueue: `iters` launches captured in one
    HIP graph, replayed `reps` times."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (reps * iters) * 1e3


TIMER = time_graph if os.environ.get("CROSS_BENCH_GRAPH") == "1" else time_fn


def main(iters=50):
    N, H, K, B = 8, 8, 77, 4
    tok = default_tokenizer()
    mapper = seq_aligner.get_replacement_mapper(pl.north_star_prompts(), tok)
    prog = programs.replace_program(mapper).to_device("cuda")
    # zero-term program: P0 recomputed and parked in the slab, no gather (isolates the gather cost)
    prog0 = programs.replace_program(torch.zeros_like(mapper)).to_device("cuda")
    alpha = torch.ones(B - 1, K, device="cuda")
    rows = []
    for name, P, d in GEOMS:
        C = H * d
        g = torch.Generator(device="cuda").manual_seed(P)
        q = torch.randn(N, P, C, device="cuda", generator=g).to(torch.bfloat16)
        k = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
        v = torch.randn(N, K, C, device="cuda", generator=g).to(torch.bfloat16)
        o = torch.empty_like(q)
        store = torch.zeros(B * H, P, K, device="cuda")
        slots = [-1] * B + [i * H for i in range(B)]
        plain = [(0, B, None, None), (B, B, None, None)]
        edit = [(0, B, None, None), (B, B, prog, alpha)]
        edit0 = [(0, B, None, None), (B, B, prog0, alpha)]
        # LocalBlend word sums folded into the store epilogue (the 16x16 layers G3/G5 in the pipeline):
        # [count, 2, lh, P] f32 running sums, alpha / substruct weights [count, K]
        lh = 5 * H
        bsums = torch.zeros(B, 2, lh, P, device="cuda")
        balpha = torch.rand(B, K, device="cuda")
        blend = [(0, B, None, None), (B, B, prog, alpha, (bsums, balpha, None, 0, lh))]
        r = {"geom": name, "P": P, "d": d}
        for tag, grp, st in (("plain", plain, None), ("edit", edit, None), ("edit_no_terms", edit0, None),
                             ("store", plain, store),
                             ("edit+store", edit, store), ("edit+store+blend", blend, store)):
            fn = lambda: _hip.cross_attn(q, k, v, o, H, d ** -0.5, grp, store=st,  # noqa: E731
                                         store_slot=slots if st is not None else None,
                                         accumulate=st is not None)
            r[tag + "_us"] = round(TIMER(fn, iters), 2)
        print(json.dumps(r), flush=True)
        rows.append(r)
    return rows


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
