"""Per-kernel stats (name, calls, total/avg ns, %) from a rocprofv3 rocpd SQLite database,
in the column layout of rocprofv3's kernel_stats.csv.  usage: rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, k, s, a, lo, hi in rows:
        w.writerow([n, k, s, round(a, 1), round(100.0 * s / total, 2), lo, hi])


if __name__ == "__main__":
    main()
