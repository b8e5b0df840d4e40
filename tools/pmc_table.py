"""Derived per-kernel PMC table from tools/gpu_pmc.sh summaries (profiles/rNN/pmc/*_summary.txt):
MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128) (the r01b convention: GRBM
sums the 8 XCDs, 1024 SIMDs), HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md HBM: the
gfx950 FETCH_SIZE halving), wave-time split (SQ_WAIT_ANY = parked on s_waitcnt / barrier,
SQ_WAIT_INST_ANY = issue stalls, SQ_ACTIVE_INST_ANY), LDS bank conflicts / LDS-active cycles.
Usage: python tools/pmc_table.py <summary.txt> <kernel substring> [<label> <algorithmic bytes>] ..."""
import sys


def load(path, sub):
    vals = {}
    for line in open(path):
        parts = line.rstrip("\n").split("\t")
        if len(parts) >= 3 and sub in parts[0]:
            vals[parts[1]] = float(parts[2])
    return vals


def row(path, sub, label, alg):
    v = load(path, sub)
    busy = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (v["GRBM_GUI_ACTIVE"] * 128)
    hbm = v["FETCH_SIZE"] * 1024 * 2 + v["WRITE_SIZE"] * 1024
    wc = v["SQ_WAVE_CYCLES"]
    return (f"| {label} | {100 * busy:.1f} % | {hbm / 1e6:.1f} MB | {alg / 1e6:.1f} MB | "
            f"{100 * v['SQ_WAIT_ANY'] / wc:.0f} % | {100 * v['SQ_WAIT_INST_ANY'] / wc:.0f} % | "
            f"{100 * v['SQ_ACTIVE_INST_ANY'] / wc:.0f} % | "
            f"{100 * v['SQ_LDS_BANK_CONFLICT'] / max(v['SQ_LDS_IDX_ACTIVE'], 1):.1f} % | "
            f"{v['SQ_INSTS_VALU'] / max(v['SQ_INSTS_MFMA'], 1):.1f} |")


if __name__ == "__main__":
    a = sys.argv[1:]
    print("| kernel | MFMA pipe busy | HBM bytes / launch (PMC) | algorithmic | wave time parked (waitcnt, barrier) "
          "| issue-stalled | issuing | LDS bank conflicts | VALU-encoded instr. per MFMA |")
    print("|---|---|---|---|---|---|---|---|---|")
    for i in range(0, len(a), 4):
        print(row(a[i], a[i + 1], a[i + 2], float(a[i + 3])))
