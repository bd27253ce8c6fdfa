"""Per-kernel statistics from a rocprofv3 SQLite (rocpd) database: the CSV that
``--stats`` writes in the csv output format.  usage: rocpd_stats.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db_path):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), "
                      "max(end - start) from kernels group by name order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    return [(n, c, t, a, 100.0 * t / total, lo, hi) for n, c, t, a, lo, hi in rows]


def main():
    rows = stats(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], round(r[3], 1), round(r[4], 2), r[5], r[6]])


if __name__ == "__main__":
    main()
