#!/usr/bin/env python3
"""rocprofv3 kernel trace CSV -> per (kernel, grid) duration summary (profiles/<round>/kernel_stats_by_grid.csv)."""
import csv
import sys


def main(src, dst):
    agg = {}
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"][:120]
        grid = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) * int(r.get("Grid_Size_Z", 1) or 1)
        key = (name, grid, int(r["Workgroup_Size_X"]), r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")),
               r.get("Scratch_Size", r.get("Private_Segment_Size", "")))
        agg.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid_lanes", "wg", "vgpr", "scratch_b", "calls", "avg_ms", "min_ms", "max_ms", "total_ms"])
        for (name, grid, wg, vgpr, scr), d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, grid, wg, vgpr, scr, len(d), "%.4f" % (sum(d) / len(d)), "%.4f" % min(d),
                        "%.4f" % max(d), "%.3f" % sum(d)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
