"""Kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite, ROCm 7): every kernel's
calls / total / average, the hot-path (libp2p_hip) kernels split by launch grid -- the same kernel
serves several U-Net geometries -- and the hot path's share of GPU kernel time.
Usage: python tools/rocpd_summary.py <run_results.db> [> summary.txt]"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, lds_size from kernels").fetchall()
    tot = sum(r[1] for r in rows)
    by = {}
    for name, dur, gx, wx, vg, lds in rows:
        by.setdefault(name, []).append(dur)
    print(f"kernels: {len(rows)} dispatches, {tot / 1e6:.3f} ms GPU kernel time")
    print("\n== top 15 kernels (all)")
    for name, ds in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:15]:
        print(f"{sum(ds) / tot * 100:6.2f}%  calls {len(ds):6d}  avg {sum(ds) / len(ds) / 1e3:9.2f} us  {name[:110]}")
    hot = [r for r in rows if "p2p" in r[0]]
    htot = sum(r[1] for r in hot)
    print(f"\n== hot path (p2p kernels): {htot / 1e6:.3f} ms = {htot / tot * 100:.2f}% of kernel time")
    grp = {}
    for name, dur, gx, wx, vg, lds in hot:
        short = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        grp.setdefault((short, gx // wx if wx else gx, wx, vg, lds), []).append(dur)
    for (short, nwg, wx, vg, lds), ds in sorted(grp.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(ds) / tot * 100:6.2f}%  calls {len(ds):6d}  avg {sum(ds) / len(ds) / 1e3:9.2f} us  "
              f"wgs {nwg:6d} x {wx:4d} thr  vgpr {vg:3d}  lds {lds:6d}  {short[:100]}")


if __name__ == "__main__":
    main(sys.argv[1])
