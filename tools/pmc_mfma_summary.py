"""MFMA-busy fraction per kernel class from a rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE CSV.

usage: python tools/pmc_mfma_summary.py <counter_collection.csv> <out.json> [n_cu]

SQ_VALU_MFMA_BUSY_CYCLES sums, over every SIMD, the cycles its matrix core is busy (16 per
v_mfma_f32_16x16x32_f16, 32 per 32x32x16: MI355X_MICROARCH.md, PMC units).  GRBM_GUI_ACTIVE is
the kernel's GPU-busy cycles summed over the 8 XCDs, so kernel cycles = GRBM_GUI_ACTIVE / 8 and
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles * n_cu * 4 SIMDs).
The effective clock (kernel cycles / kernel wall time) is reported when the CSV carries timestamps.
GRBM_GUI_ACTIVE also counts cycles outside a short dispatch's own span (round 5 printed 2.4-14.9 GHz for
kernels under ~0.3 ms, above the 2.4 GHz the chip can run): the kernel cycles are therefore capped at
wall time x 2.4 GHz (so a short kernel's busy fraction is not deflated by the inflated denominator),
and the clock is reported only for classes whose dispatches average >= 0.3 ms; below that it is null.
The authoritative clock is the in-kernel s_memtime / s_memrealtime measurement of tools/clock_probe.py
(profiles/r06_clock_probe.log: fc1 1.74 GHz, spatial attention 1.69 GHz)."""
import csv, json, re, sys
from collections import defaultdict

# Stable tags of the forward's kernel classes (the demangled names carry template arguments that change
# as kernels evolve; bench.py looks its figures up by tag).  Template arguments of gemm256_kernel:
# <XR, WR, CONV, ACT, ROWB, LNF, EK>; ACT 1 = GELU; LNF = LayerNorm folded into the epilogue.
TAGS = [
    (r"^gemm256_kernel<2, 2, false, 1, false, true\b", "enc_fc1"),            # norm2 + fc1 + GELU (register epilogue)
    (r"^gemm256_kernel<2, 2, false, 0, false, true, 1>", "enc_qkv"),          # norm1 + qkv (register epilogue)
    (r"^gemm256_kernel<2, 2, false, 0, false, true, 3>", "mm_qkv_lnfold"),    # motion-module LN + q/k/v + PE
    (r"^gemm256_kernel<2, 2, false, 0, false, false, 0>", "gemm_staged"),      # proj / fc2 (+ residual, row stats) and others
    (r"^gemm256_kernel<2, 2, false, 0, false, false, 1>", "gemm_bias_rows"),
    (r"^gemm256_kernel<2, 2, false, 0, true\b", "gemm_rowbias"),
    (r"^gemm256_kernel<2, 2, false, 2\b", "gemm_geglu"),
    (r"^gemm256_kernel<2, 2, true\b", "conv_phased"),
    (r"spatial_attn32_kernel", "spatial_attention"),
    (r"temporal_attn_lds_kernel", "temporal_attention"),
    (r"depth_conv_kernel", "depth_conv"),
    (r"halo_conv_kernel<64, 128, 1|halo_conv_kernelILi64ELi128ELi1E", "output_conv1"),
    (r"^hconv256_kernel", "conv3x3_halo256"),
    (r"^strip_conv", "conv3x3_strip"),
]


def tag_of(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", name)  # mangled anonymous-namespace kernels
    for rx, t in TAGS:
        if re.search(rx, name):
            return t
    return None


path, out = sys.argv[1], sys.argv[2]
n_cu = int(sys.argv[3]) if len(sys.argv) > 3 else 256
disp = defaultdict(dict)
for r in csv.DictReader(open(path)):
    d = disp[r["Dispatch_Id"]]
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    d["name"] = re.sub(r"\(.*", "", name)[:70]
    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    if "Start_Timestamp" in r and r.get("End_Timestamp"):
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
agg = defaultdict(lambda: {"dispatches": 0, "mfma_busy_cycles": 0.0, "kernel_cycles": 0.0, "ns": 0})
for d in disp.values():
    if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
        continue
    a = agg[d["name"]]
    a["dispatches"] += 1
    a["mfma_busy_cycles"] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
    cyc = d["GRBM_GUI_ACTIVE"] / 8.0
    if d.get("ns"):
        cyc = min(cyc, d["ns"] * 2.4)  # no more than the wall time at the 2.4 GHz maximum clock
    a["kernel_cycles"] += cyc
    a["grbm_cycles"] = a.get("grbm_cycles", 0.0) + d["GRBM_GUI_ACTIVE"] / 8.0
    a["ns"] += d.get("ns", 0)
res = {"n_cu": n_cu, "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (min(GRBM_GUI_ACTIVE/8, wall ns x 2.4) * n_cu * 4)",
       "kernels": {}}
tot_b = tot_c = tot_g = 0.0
for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["kernel_cycles"]):
    busy = a["mfma_busy_cycles"] / max(1.0, a["kernel_cycles"] * n_cu * 4)
    e = {"tag": tag_of(k), "dispatches": a["dispatches"], "mfma_busy": round(busy, 4), "kernel_cycles": a["kernel_cycles"]}
    if a["ns"]:
        long_enough = a["ns"] / a["dispatches"] >= 300e3
        e["clock_ghz"] = round(a["grbm_cycles"] / a["ns"], 3) if long_enough else None
        e["mean_dispatch_us"] = round(a["ns"] / a["dispatches"] / 1e3, 1)
    res["kernels"][k] = e
    tot_b += a["mfma_busy_cycles"]
    tot_c += a["kernel_cycles"]
    tot_g += a.get("grbm_cycles", 0.0)
res["all_kernels_mfma_busy"] = round(tot_b / max(1.0, tot_c * n_cu * 4), 4)
res["all_kernels_mfma_busy_uncapped"] = round(tot_b / max(1.0, tot_g * n_cu * 4), 4)  # GRBM/8 cycles (rounds <= 5)
json.dump(res, open(out, "w"), indent=1)
for k, e in list(res["kernels"].items())[:14]:
    clk = e.get("clock_ghz")
    print(f"{e['mfma_busy']:7.3f}  {clk if clk is not None else '  -  '} GHz  {e['dispatches']:5d}  {k}")
print("all kernels", res["all_kernels_mfma_busy"], "(uncapped GRBM cycles:", res["all_kernels_mfma_busy_uncapped"], ")")
