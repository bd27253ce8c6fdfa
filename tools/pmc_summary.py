"""Per-kernel PMC summary from rocprofv3 rocpd databases: for each kernel whose name matches
a filter, the mean per dispatch of every collected counter plus the mean duration.
usage: pmc_summary.py FILTER DB [DB ...]"""
import sqlite3
import sys
from collections import defaultdict


def main():
    flt, dbs = sys.argv[1], sys.argv[2:]
    acc = defaultdict(lambda: defaultdict(list))
    for db in dbs:
        c = sqlite3.connect(db)
        for name, grid, counter, value, dur, disp in c.execute(
                "select kernel_name, grid_size, counter_name, value, duration, dispatch_id from counters_collection"):
            if flt in name:
                key = f"{name[:70]} grid={grid}"
                acc[key][counter].append(value)
                acc[key]["_dur_ns"].append(dur)
    for k, cs in acc.items():
        print(k)
        for cn in sorted(cs):
            v = cs[cn]
            print(f"   {cn:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
