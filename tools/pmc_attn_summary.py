"""Summarise tools/pmc_attn3.sh's two PMC passes per library (tuning tool): where a spatial-attention
wave's cycles go and the issue mix per MFMA.  usage: python tools/pmc_attn_summary.py TAG ...
(reads gpurun_out/pw_<TAG>_a / _b / run_counter_collection.csv; medians over the dispatches)."""
import csv
import statistics
import sys


def load(path):
    per = {}
    for r in csv.DictReader(open(path)):
        if "spatial_attn" not in r.get("Kernel_Name", ""):
            continue
        d = per.setdefault(r["Dispatch_Id"], {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    keys = set().union(*per.values()) if per else set()
    return {k: statistics.median(d.get(k, 0.0) for d in per.values()) for k in keys}


for tag in sys.argv[1:]:
    a = load(f"gpurun_out/pw_{tag}_a/run_counter_collection.csv")
    b = load(f"gpurun_out/pw_{tag}_b/run_counter_collection.csv")
    wc = a.get("SQ_WAVE_CYCLES", 1.0)
    mf = b.get("SQ_INSTS_MFMA", 1.0)
    out = {
        "wait_any (parked: waitcnt / barrier)": a.get("SQ_WAIT_ANY", 0) / wc,
        "wait_inst_any (ready, not issued)": a.get("SQ_WAIT_INST_ANY", 0) / wc,
        "wait_inst_lds": a.get("SQ_WAIT_INST_LDS", 0) / wc,
        "active_inst_valu": a.get("SQ_ACTIVE_INST_VALU", 0) / wc,
        "active_inst_lds": a.get("SQ_ACTIVE_INST_LDS", 0) / wc,
        "lds_bank_conflict / wave_cycles": a.get("SQ_LDS_BANK_CONFLICT", 0) / wc,
        "VALU per MFMA": b.get("SQ_INSTS_VALU", 0) / mf,
        "LDS per MFMA": b.get("SQ_INSTS_LDS", 0) / mf,
        "SALU per MFMA": b.get("SQ_INSTS_SALU", 0) / mf,
        "mfma_busy / (grbm/8 * 1024 SIMDs)": b.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (b.get("GRBM_GUI_ACTIVE", 1) / 8 * 1024),
        "coexec / mfma_busy": b.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0) / max(b.get("SQ_VALU_MFMA_BUSY_CYCLES", 1), 1),
    }
    print(tag + ": " + ", ".join(f"{k} {v:.3f}" for k, v in out.items()), flush=True)
