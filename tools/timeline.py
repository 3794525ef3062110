#!/usr/bin/env python3
"""Print a per-dispatch timeline from a rocprofv3 kernel-trace CSV: the dispatches between two
occurrences of a marker kernel (one pipeline step), with start offsets, durations, queue, VGPRs and
scratch.  Usage: timeline.py kt_kernel_trace.csv [--marker k_classify] [--occurrence -1] [--grid N]"""
import argparse
import csv


def base(name):
    name = name.split("(", 1)[0].strip()
    return name[5:] if name.startswith("void ") else name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="k_classify")
    ap.add_argument("--occurrence", type=int, default=-1, help="which marker occurrence starts the step")
    ap.add_argument("--before", type=int, default=4, help="dispatches shown before the marker")
    ap.add_argument("--grid", type=int, default=0, help="only markers with this grid size")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if base(r["Kernel_Name"]) == a.marker and
             (not a.grid or int(r["Grid_Size_X"]) == a.grid)]
    if not marks:
        raise SystemExit("marker not found")
    k = a.occurrence if a.occurrence >= 0 else len(marks) + a.occurrence
    lo = max(0, marks[k] - a.before)
    hi = marks[k + 1] - a.before if k + 1 < len(marks) else len(rows)
    t0 = int(rows[lo]["Start_Timestamp"])
    end = 0
    for r in rows[lo:hi]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        end = max(end, e)
        print("%9.3f %8.3f ms  q%-3s vgpr %3s scr %5s grid %9s  %s" % ((s - t0) / 1e6, (e - s) / 1e6, r["Queue_Id"],
              r["VGPR_Count"], r["Scratch_Size"], r["Grid_Size_X"], base(r["Kernel_Name"])[:70]))
    print("span %.3f ms" % ((end - t0) / 1e6))


if __name__ == "__main__":
    main()
