"""Summarise a rocprofv3 kernel-trace CSV of `bench.py --steps S --warmup 1`: per-kernel time
over the TIMED edit groups only (everything after the warm-up group), plus group wall time."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
g1 = [r for r in rows if "self_attn_fused_kernel" in r["Kernel_Name"] and ", 40," in r["Kernel_Name"]]
per_group = 250                         # 5 G1/G7 launches per U-Net call x 50 steps
n_groups = len(g1) // per_group
start = int(g1[per_group]["Start_Timestamp"]) - 3_000_000 if n_groups > 1 else int(rows[0]["Start_Timestamp"])
timed = [r for r in rows if int(r["Start_Timestamp"]) >= start]
t0 = int(timed[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in timed)
agg = collections.defaultdict(lambda: [0, 0])
for r in timed:
    agg[r["Kernel_Name"]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[r["Kernel_Name"]][1] += 1
busy = sum(v[0] for v in agg.values())
groups = max(n_groups - 1, 1)
print(f"timed groups: {groups}; wall (first..last kernel) {(t1 - t0) / 1e6:.1f} ms; kernel busy {busy / 1e6:.1f} ms; "
      f"kernels {sum(v[1] for v in agg.values())}")
print(f"{'total_ms':>10} {'calls':>7} {'avg_us':>9} {'share':>6}  kernel")
for name, (ns, calls) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:40]:
    print(f"{ns / 1e6:10.2f} {calls:7d} {ns / calls / 1e3:9.1f} {100 * ns / busy:5.1f}%  {name[:150]}")
p2p = {k: v for k, v in agg.items() if "p2p::" in k}
print(f"\np2p kernels (hot path): {sum(v[0] for v in p2p.values()) / 1e6:.1f} ms of {busy / 1e6:.1f} ms busy "
      f"({100 * sum(v[0] for v in p2p.values()) / busy:.1f}%)")
