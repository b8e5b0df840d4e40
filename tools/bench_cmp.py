"""Compare bench.py JSON lines (gpurun_out/<tag>/bench.json): headline, dominant kernel, clock and
every attention geometry's average launch, side by side.  Usage: python tools/bench_cmp.py tag1 tag2 .."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rows = {}
heads = []
for tag in sys.argv[1:]:
    f = tag if tag.endswith(".json") else os.path.join(ROOT, "gpurun_out", tag, "bench.json")
    d = json.load(open(f))
    r, a = d["roofline"], d["roofline_attn_total"]
    heads.append((tag, d["value"], r["avg_launch_ms"] * 1e3, r["frac"], r.get("sclk_mhz"), r.get("frac_at_measured_clock"),
                  a["frac"], a["by_kind"]["self"]["frac"], a["by_kind"]["cross"]["ms_per_unet_call"] * 1e3,
                  a["by_kind"]["cross"]["frac"]))
    for g in a["by_geometry"]:
        rows.setdefault(g["geometry"], []).append(g["avg_launch_ms"] * 1e3)
print(f"{'tag':24s} {'value':>7s} {'G1 us':>7s} {'frac':>6s} {'sclk':>6s} {'f@clk':>6s} {'attn':>6s} {'self':>6s} "
      f"{'x us/c':>7s} {'x hbm':>6s}")
for h in heads:
    print(f"{h[0]:24s} {h[1]:7.4f} {h[2]:7.2f} {h[3]:6.4f} {h[4] or 0:6.0f} {h[5] or 0:6.4f} {h[6]:6.4f} {h[7]:6.4f} "
          f"{h[8]:7.1f} {h[9]:6.4f}")
for geo, vals in rows.items():
    print(f"  {geo:20s} " + " ".join(f"{x:7.2f}" for x in vals))
