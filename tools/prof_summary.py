"""Summarise a rocprofv3 run (rocpd SQLite db or kernel_stats.csv) into a
per-kernel table: calls, total/avg/min/max duration (us), share of GPU time.

Usage: python tools/prof_summary.py gpurun_out/prof/run_results.db > profiles/rNN_name.txt
"""
import csv
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by sum(end-start) desc").fetchall()
    return [(n.split("(")[0], k, t / 1e3, a / 1e3, mn / 1e3, mx / 1e3) for n, k, t, a, mn, mx in rows]


def from_csv(path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"].split("(")[0], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                    float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    return out


def main():
    p = sys.argv[1]
    rows = from_db(p) if p.endswith(".db") else from_csv(p)
    tot = sum(r[2] for r in rows) or 1.0
    print("# rocprofv3 --kernel-trace --stats summary of %s" % os.path.basename(p))
    print("%-28s %6s %12s %11s %11s %11s %7s" % ("kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"))
    for n, k, t, a, mn, mx in rows:
        print("%-28s %6d %12.1f %11.2f %11.2f %11.2f %6.2f%%" % (n[:28], k, t, a, mn, mx, 100 * t / tot))


if __name__ == "__main__":
    main()
