"""Kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite, ROCm 7): every kernel's
calls / total / average, the hot-path (libp2p_hip) kernels split by launch grid -- the same kernel
serves several U-Net geometries -- and the hot path's share of GPU kernel time.
With --split-last N: the dominant hot-path kernel's launches split in dispatch order -- the last N
(bench.py's eager per-launch timing pass after a graphed timed region) against the rest (warm-up and
graph replays) --, each without the launches that ran beside a clock probe (bench.py's ClockProbe:
those lose 8 CUs and leave the bench's averages too).
Usage: python tools/rocpd_summary.py <run_results.db> [--split-last N] [> summary.txt]"""
import sqlite3
import sys


def split_last(c, n_last):
    """The dominant p2p kernel's average, probed launches excluded, over its last n_last dispatches
    and over the others."""
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    hot = {}
    for name, st, en, dur in rows:
        if "p2p" in name:
            hot[name] = hot.get(name, 0) + dur
    dom = max(hot, key=hot.get)
    probes = [(st, en) for name, st, en, _ in rows if "clock_probe_kernel" in name]
    launches = [(st, en, dur) for name, st, en, dur in rows if name == dom]

    def probed(st, en):
        return any(ps < en and pe > st for ps, pe in probes)
    marks = [(dur, probed(st, en)) for st, en, dur in launches]
    last, rest = marks[-n_last:], marks[:-n_last]

    def avg(part):
        clean = [d for d, p in part if not p]
        return (sum(clean) / len(clean) / 1e3 if clean else float("nan")), len(clean), len(part) - len(clean)
    short = dom.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    print(f"\n== dominant kernel by dispatch order: {short[:90]}")
    for label, part in (("last %d (eager timing pass)" % n_last, last), ("the rest (warm-up, graph replays)", rest),
                        ("all", marks)):
        a, n, p = avg(part)
        print(f"  {label:40s} avg {a:8.2f} us over {n} launches ({p} beside a clock probe left out)")


def main(path, n_last=0):
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


    if n_last:
        split_last(c, n_last)


if __name__ == "__main__":
    args = sys.argv[1:]
    n = 0
    if "--split-last" in args:
        i = args.index("--split-last")
        n = int(args[i + 1])
        del args[i:i + 2]
    main(args[0], n)
