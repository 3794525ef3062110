"""Per-kernel summary (calls, avg, total) from a rocprofv3 SQLite output, plus a per-dispatch
timeline of one kernel family when asked:  python tools/kstats_db.py <db> [name-substring]"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute("select %s, start, end, stream_id from kernels order by start" % name).fetchall()
    agg = {}
    for n, s, e, _ in rows:
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
    for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
        print("%-70s %5d %9.3f ms avg %9.3f ms tot" % (n[:70], k, t / k / 1e6, t / 1e6))
    if len(sys.argv) > 2:
        t0 = None
        for n, s, e, sid in rows:
            if sys.argv[2] in n:
                t0 = s if t0 is None else t0
                print("%9.3f %9.3f  s%-3s %s" % ((s - t0) / 1e6, (e - s) / 1e6, sid, n[:70]))


if __name__ == "__main__":
    main()
