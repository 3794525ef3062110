"""Condense rocprofv3 --pmc counter_collection CSVs (one row per dispatch and counter) into one row per
(kernel, grid, counter): the mean value per dispatch and the dispatch count.  The output keeps the
columns bench.py's profile_traffic() reads (Kernel_Name, Grid_Size, Counter_Name, Counter_Value).

    python tools/pmc_summary.py <counter_collection.csv> <out.csv>
"""
import csv
import sys


def base(name):
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    name = name.replace("(anonymous namespace)::", "")
    return name.split("(", 1)[0].strip()


def main():
    agg = {}
    with open(sys.argv[1], newline="") as f:
        for r in csv.DictReader(f):
            key = (base(r["Kernel_Name"]), int(r["Grid_Size"]), r["Counter_Name"])
            a = agg.setdefault(key, [0.0, 0])
            a[0] += float(r["Counter_Value"])
            a[1] += 1
    with open(sys.argv[2], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value", "Dispatches"])
        for (k, g, c), (s, n) in sorted(agg.items()):
            w.writerow([k, g, c, "%.3f" % (s / n), n])


if __name__ == "__main__":
    main()
