"""Kernel statistics (name, calls, total/avg/min/max ns) from a rocprofv3 SQLite output
(run_results.db, the default format of ROCm 7.2's rocprofv3), in the column layout of
its --stats kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/X/run_results.db [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import sys


def stats(db: str):
    con = sqlite3.connect(db)
    rows = con.execute("SELECT name, COUNT(*), SUM(end - start), AVG(end - start), MIN(end - start), "
                       "MAX(end - start) FROM kernels GROUP BY name ORDER BY SUM(end - start) DESC").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [dict(Name=r[0], Calls=r[1], TotalDurationNs=r[2], AverageNs=r[3], MinNs=r[4], MaxNs=r[5],
                 Percentage=100.0 * r[2] / tot) for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    a = ap.parse_args()
    st = stats(a.db)
    out = open(a.csv, "w", newline="") if a.csv else sys.stdout
    w = csv.DictWriter(out, fieldnames=list(st[0].keys()) if st else ["Name"])
    w.writeheader()
    for r in st:
        w.writerow(r)


if __name__ == "__main__":
    main()
