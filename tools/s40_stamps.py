"""Where a wave of the d = 40 self-attention kernel spends its cycles (experiments build, variant
163 = the production shape with s_memtime stamps): prologue, per-tile compute, barrier wait per
tile, recompute check + epilogue, and the launch timeline.  Stamps of the first S40_NWG (512) workgroups of a config-2 G1
launch (N = 8, H = 8, P = K = 4096, d = 40).
Usage: P2P_EXPERIMENTS_LIB=1 P2P_SELF_VARIANT=163 python tools/s40_stamps.py
       S40_STAMPS=P,d,waves,bk,qb (default 4096,40,8,256,2; the d = 80 stamped variant 103:
       S40_STAMPS=1024,80,4,128,2)"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "prompt-to-prompt_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from p2p_amd import _hip  # noqa: E402

SLOTS, NWG = 40, int(os.environ.get("S40_NWG", "512"))
P, D, WAVES, BK, QB = (int(x) for x in os.environ.get("S40_STAMPS", "4096,40,8,256,2").split(","))
NTILES = P // BK
X = (BK // 32) * QB   # 32x32 blocks per tile per wave


def main():
    N, H, P_, d = 8, 8, P, D
    C = H * d
    q = torch.randn(N, P_, C, device="cuda").to(torch.bfloat16)
    k = torch.randn(N, P_, C, device="cuda").to(torch.bfloat16)
    v = torch.randn(N, P_, C, device="cuda").to(torch.bfloat16)
    o = torch.empty_like(q)
    for _ in range(20):
        _hip.self_attn(q, k, v, o, H, d ** -0.5)
    torch.cuda.synchronize()
    buf = np.zeros(NWG * WAVES * SLOTS, dtype=np.uint64)
    fn = _hip.lib().p2p_diag_self40_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
    rc = fn(buf.ctypes.data, buf.nbytes)
    assert rc == 0, rc
    st = buf.reshape(NWG, WAVES, SLOTS).astype(np.int64)
    t0 = st[:, :, 0]
    pro = st[:, :, 1] - t0
    comp, bar = [], []
    prev = st[:, :, 1]
    for kt in range(NTILES):
        e, b = st[:, :, 2 + 2 * kt], st[:, :, 3 + 2 * kt]
        comp.append(e - prev)
        bar.append(b - e)
        prev = b
    comp, bar = np.stack(comp, -1), np.stack(bar, -1)
    chk = st[:, :, 36] - prev
    epi = st[:, :, 37] - st[:, :, 36]
    tot = st[:, :, 37] - t0
    med = lambda a: float(np.median(a))  # noqa: E731
    print(f"cycles per wave (median over {NWG} workgroups x {WAVES} waves):")
    print(f"  total {med(tot):.0f}  prologue {med(pro):.0f}  compute/tile {med(comp):.0f} (x{NTILES} = {med(comp.sum(-1)):.0f})"
          f"  barrier/tile {med(bar):.0f} (x{NTILES} = {med(bar.sum(-1)):.0f})  check {med(chk):.0f}  epilogue {med(epi):.0f}")
    print(f"  compute per 32x32 block: {med(comp) / X:.0f} cycles per wave")
    print(f"  tile 0 compute {med(comp[..., 0]):.0f}, tiles 1-{NTILES - 1} {med(comp[..., 1:]):.0f}")
    # younger half vs older half
    print(f"  older half compute/tile {med(comp[:, :WAVES // 2]):.0f} barrier/tile {med(bar[:, :WAVES // 2]):.0f};"
          f" younger half compute/tile {med(comp[:, WAVES // 2:]):.0f} barrier/tile {med(bar[:, WAVES // 2:]):.0f}")
    # skew of barrier arrival within a workgroup
    arr = st[:, :, 2:2 + 2 * NTILES:2]
    skew = arr.max(1) - arr.min(1)
    print(f"  arrival skew per tile (max-min over the waves): median {med(skew):.0f}, p90 {float(np.percentile(skew, 90)):.0f}")
    # launch timeline (s_memrealtime, 100 MHz): workgroup busy time against the launch span
    rs, re_ = st[:, 0, 38], st[:, 0, 39]
    span = (re_.max() - rs.min()) * 10.0   # ns
    busy = float(((re_ - rs) * 10.0).sum())
    ncu = 256
    print(f"  timeline: span {span / 1e3:.1f} us, workgroup time summed {busy / 1e3:.1f} us over {NWG} workgroups;"
          f" busy fraction of {ncu} CUs {busy / (ncu * span):.3f}; per-workgroup median {med((re_ - rs) * 10.0) / 1e3:.2f} us")
    order = np.argsort(rs)
    rel = (rs[order] - rs.min()) * 10.0 / 1e3
    print("  start times (us) by rank: " + " ".join(f"{rel[i]:.1f}" for i in (0, 64, 128, 255, 256, 320, 384, 448, NWG - 1) if i < NWG))
    ends = np.sort((re_ - rs.min()) * 10.0 / 1e3)
    print("  end times (us) by rank: " + " ".join(f"{ends[i]:.1f}" for i in (0, 64, 128, 255, 256, 320, 384, 448, NWG - 1) if i < NWG))
    start_skew = t0.max(1) - t0.min(1)
    print(f"  workgroup start skew {med(start_skew):.0f}; workgroups' start spread {float(t0[:, 0].max() - t0[:, 0].min()):.0f}")


if __name__ == "__main__":
    main()
