"""VALU issue model per kernel from one rocprofv3 --pmc pass that holds SQ_INSTS_VALU and GRBM_GUI_ACTIVE
(tools/profile.sh pass `issue`): per (kernel, grid) the mean over its dispatches of

    duration_ms        End - Start of the dispatch (the PMC pass serialises kernels)
    valu_per_launch    SQ_INSTS_VALU (wave-instructions)
    eff_clock_ghz      GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md: the counter sums the 8 XCDs)
    cyc_per_valu       (GRBM_GUI_ACTIVE / 8) / (SQ_INSTS_VALU / 1024 SIMDs): shader-clock cycles per VALU
                       wave-instruction per SIMD.  tools/microbench_valu.hip measures ~2.3-2.6 for the
                       dual-issue ops (add/sub/and/or/xor/mov/lshrrev/bitop3/fma_f32) and ~4.2 for every
                       other VALU opcode with >= 2 waves per SIMD (profiles/r04/microbench_valu*.txt), so a
                       kernel at ~4.2 is issue-bound on its instruction count.

    python tools/issue_summary.py <counter_collection.csv> <out.csv>
"""
import csv
import sys

SIMDS = 1024
XCDS = 8


def base(name):
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    return name.replace("(anonymous namespace)::", "").split("(", 1)[0].strip()


def main():
    disp = {}
    with open(sys.argv[1], newline="") as f:
        for r in csv.DictReader(f):
            key = (base(r["Kernel_Name"]), int(r["Grid_Size"]))
            d = disp.setdefault(key, {}).setdefault(r["Dispatch_Id"], {
                "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), "vgpr": r.get("VGPR_Count", ""),
                "scratch": r.get("Scratch_Size", "")})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    rows = []
    for (k, g), ds in sorted(disp.items()):
        ds = [d for d in ds.values() if "SQ_INSTS_VALU" in d and "GRBM_GUI_ACTIVE" in d and d["ns"] > 0]
        if not ds:
            continue
        n = len(ds)
        ns = sum(d["ns"] for d in ds) / n
        valu = sum(d["SQ_INSTS_VALU"] for d in ds) / n
        grbm = sum(d["GRBM_GUI_ACTIVE"] for d in ds) / n
        waves = sum(d.get("SQ_WAVES", 0.0) for d in ds) / n
        clk = grbm / XCDS / ns
        cpi = (grbm / XCDS) / (valu / SIMDS) if valu else 0.0
        rows.append([k, g, n, "%.4f" % (ns * 1e-6), "%.0f" % valu, "%.0f" % waves,
                     "%.1f" % (valu / waves) if waves else "", "%.3f" % clk, "%.3f" % cpi, ds[0]["vgpr"],
                     ds[0]["scratch"]])
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size", "Dispatches", "Duration_ms", "VALU_per_launch", "Waves",
                    "VALU_per_wave", "Eff_clock_GHz", "Cyc_per_VALU_per_SIMD", "VGPR_Count", "Scratch_Size"])
        w.writerows(rows)


if __name__ == "__main__":
    main()
