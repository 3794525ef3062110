#!/usr/bin/env python3
"""Kernels + memory copies of one step from a rocprofv3 trace directory, in start order, from the last
dispatch whose name contains --marker: start offset, duration, queue, VGPRs, scratch, grid, name.
Usage: kt_timeline.py <trace dir> [--marker k_stx_parse<false>] [--count 60]"""
import argparse
import csv
import glob
import os


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()[:64]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="k_stx_parse<false>")
    ap.add_argument("--count", type=int, default=60)
    ap.add_argument("--occurrence", type=int, default=-1)
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(kt)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if not idx:
        raise SystemExit("marker not found")
    i0 = idx[a.occurrence]
    t0 = int(rows[i0]["Start_Timestamp"])
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "q%-3s v%-3s s%-4s g%-9s %s" % (
        r["Queue_Id"], r["VGPR_Count"], r["Scratch_Size"], r["Grid_Size_X"], short(r["Kernel_Name"]))) for r in rows[i0:]]
    mc = glob.glob(os.path.join(a.dir, "**", "*memory_copy_trace.csv"), recursive=True)
    if mc:
        for r in csv.DictReader(open(mc[0])):
            if int(r["Start_Timestamp"]) >= t0:
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy %s" % r.get("Direction", "")))
    ev.sort()
    for s, e, n in ev[:a.count]:
        print("%9.3f %8.3f  %s" % ((s - t0) / 1e6, (e - s) / 1e6, n))


if __name__ == "__main__":
    main()
