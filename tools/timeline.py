"""One cfg2 step's kernel timeline from a rocprofv3 --kernel-trace CSV: the last complete step (delimited by
k_ed_comb_finish launches), each kernel's start / end relative to the step's first kernel and the idle gaps
on the device.   python tools/timeline.py <kernel_trace.csv>"""
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r.get("Queue_Id", 0) or 0)))
    rows.sort()
    fin = [i for i, r in enumerate(rows) if r[2] == "k_ed_comb_finish"]
    if len(fin) < 3:
        print("need 3 steps")
        return
    a, b = fin[-3] + 1, fin[-2] + 1   # kernels after the previous finish up to this step's finish
    # include the bitmap after the finish
    while b < len(rows) and rows[b][2] in ("k_bitmap", "k_ed25519_verify"):
        b += 1
    t0 = rows[a][0]
    busy_end = t0
    for s, e, n, q in rows[a:b]:
        gap = max(0, s - busy_end)
        print("%8.1f %8.1f %7.1f  gap %6.1f  q%d %s" % ((s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3, gap / 1e3, q, n))
        busy_end = max(busy_end, e)
    print("step span %.1f us" % ((busy_end - t0) / 1e3))


if __name__ == "__main__":
    main()
