"""Kernel statistics from a rocprofv3 database (run_results.db, the default
output format of this rocprofv3) in the shape of its --stats CSV:
Name,Calls,TotalDurationNs,AverageNs,Percentage.
usage: python tools/rocpd_stats.py <run_results.db> <out.csv>
"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for r in rows:
            w.writerow(r)
    for r in rows[:8]:
        print(r)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
