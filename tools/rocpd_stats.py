"""Kernel statistics (the rocprofv3 --stats table: calls, total / average / min / max ns, share) from a rocprofv3
rocpd SQLite database (rocprofv3 7.x writes run_results.db unless --output-format csv).

  python3 tools/rocpd_stats.py DB [--csv OUT]
"""
import argparse
import csv
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                       "from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(n, c, t, a, lo, hi, 100.0 * t / total) for n, c, t, a, lo, hi in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    st = stats(a.db)
    out = open(a.csv, "w", newline="") if a.csv else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in st:
        w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", r[4], r[5], f"{r[6]:.2f}"])


if __name__ == "__main__":
    main()
