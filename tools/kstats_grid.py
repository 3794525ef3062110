"""Per-(kernel, grid) statistics from a rocprofv3 --kernel-trace CSV, so every roofline fraction in
the bench line can be recomputed from the committed profile alone (a kernel launched over several
configurations has one row per grid size).

    python tools/kstats_grid.py <kt_kernel_trace.csv> [out.csv]
"""
import csv
import sys


def main():
    src = sys.argv[1]
    agg = {}
    with open(src, newline="") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
            ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            key = (name, grid, wg, r["VGPR_Count"], r["Scratch_Size"])
            a = agg.setdefault(key, [0, 0, None, 0])
            a[0] += 1
            a[1] += ns
            a[2] = ns if a[2] is None else min(a[2], ns)
            a[3] = max(a[3], ns)
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    hdr = ["kernel", "grid_lanes", "wg", "vgpr", "scratch_b", "calls", "avg_ms", "min_ms", "max_ms", "total_ms"]
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(hdr)
    for (name, grid, wg, vgpr, scr), (k, tot, mn, mx) in rows:
        w.writerow([name[:120], grid, wg, vgpr, scr, k, "%.4f" % (tot / k / 1e6), "%.4f" % (mn / 1e6),
                    "%.4f" % (mx / 1e6), "%.3f" % (tot / 1e6)])


if __name__ == "__main__":
    main()
