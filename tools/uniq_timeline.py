"""Kernel timeline of the last full-size uniqueness commit in a rocprofv3 kernel-trace CSV:
python tools/uniq_timeline.py <kt_kernel_trace.csv> [min_grid]"""
import csv
import sys

rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:44], int(r["Grid_Size_X"])))
rows.sort()
mg = int(sys.argv[2]) if len(sys.argv) > 2 else 9_000_000
idx = [i for i, r in enumerate(rows) if r[2].startswith("k_uniq_lookup") and r[3] >= mg]
i0 = idx[-1]
t0 = rows[i0 - 3][0]
for r in rows[i0 - 3:]:
    print("%9.3f %8.3f %-44s %d" % ((r[0] - t0) / 1e6, (r[1] - r[0]) / 1e6, r[2], r[3]))
    if r[2].startswith("k_uniq_status"):
        print("total %.3f ms" % ((r[1] - t0) / 1e6))
        break
