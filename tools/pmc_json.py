"""Build profiles/<round>/pmc_g1.json (what bench.py reports as roofline.traffic) from a
tools/gpu_pmc.sh summary: FETCH_SIZE x2 (gfx950: it reports half the bytes of 16-B-per-lane
streaming reads, MI355X_MICROARCH.md HBM) + WRITE_SIZE, per launch of the dominant kernel.
Usage: python tools/pmc_json.py <summary.txt> <kernel-substring> <out.json> <kernel label>"""
import json
import sys


def main(summary, sub, out, label):
    vals = {}
    for line in open(summary):
        parts = line.rstrip("\n").split("\t")
        if len(parts) < 3 or sub not in parts[0]:
            continue
        vals[parts[1]] = float(parts[2])
    fetch_kb, write_kb = vals["FETCH_SIZE"], vals["WRITE_SIZE"]
    rd, wr = fetch_kb * 1024 * 2, write_kb * 1024
    d = {"kernel": label,
         "command": "rocprofv3 --pmc <counters> -- python3 tools/g1_only.py 20 (tools/gpu_pmc.sh; one pass per "
                    "counter group; mean over dispatches 2..20)",
         "FETCH_SIZE_kB": fetch_kb, "WRITE_SIZE_kB": write_kb,
         "fetch_correction": "x2 (MI355X_MICROARCH.md HBM: FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads)",
         "hbm_read_bytes": rd, "hbm_write_bytes": wr, "traffic_bytes_per_launch": rd + wr,
         "algorithmic_bytes_per_launch": 4 * 8 * 4096 * 320 * 2}
    for k in ("SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_WAVE_CYCLES",
              "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
              "SQ_INSTS_LDS", "SQ_ACTIVE_INST_VALU", "SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_LDS"):
        if k in vals:
            d[k] = vals[k]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
        d["mfma_pipe_busy_frac"] = vals["SQ_VALU_MFMA_BUSY_CYCLES"] / (vals["GRBM_GUI_ACTIVE"] * 128)
        d["mfma_pipe_busy_note"] = "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128), the r01b convention"
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main(*sys.argv[1:5])
