"""Per-kernel L2 <-> fabric bytes from rocprofv3 counter CSVs (FETCH_SIZE / WRITE_SIZE, KB
per dispatch) of a one-lane bench run: the last batch (from its preprocess kernel), bytes
per kernel, achieved GB/s against the kernel's duration, and the batch total.
usage: tcc_bytes.py fetch_dir write_dir"""
import csv
import glob
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    rows = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        key = int(r["Dispatch_Id"])
        rows.setdefault(key, [r["Kernel_Name"], 0.0, int(r.get("End_Timestamp") or 0) - int(r.get("Start_Timestamp") or 0)])
        rows[key][1] += float(r["Counter_Value"])
    return rows


def last_batch(rows, marker="preprocess"):
    ids = sorted(rows)
    starts = [i for i in ids if marker in rows[i][0]]
    s = starts[-1]
    # chunked head: up to 4 preprocess launches per batch; start at the first of the last group
    while starts and len(starts) > 1 and starts[-2] >= s - 4:
        s = starts[-2]
        starts = starts[:-1]
    return [i for i in ids if i >= s]


def _short(name: str) -> str:
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    ids_f = last_batch(fetch)
    ids_w = last_batch(write)
    agg = defaultdict(lambda: [0.0, 0.0, 0])
    for i in ids_f:
        n = _short(fetch[i][0])
        agg[n][0] += fetch[i][1] * 1024
        agg[n][2] += 1
    for i in ids_w:
        n = _short(write[i][0])
        agg[n][1] += write[i][1] * 1024
    tot_r = sum(v[0] for v in agg.values())
    tot_w = sum(v[1] for v in agg.values())
    print(f"{'kernel':72s} {'n':>3s} {'read MB':>9s} {'write MB':>9s}")
    for k, (r, w, n) in sorted(agg.items(), key=lambda kv: -(kv[1][0] + kv[1][1])):
        print(f"{k:72s} {n:3d} {r / 1e6:9.1f} {w / 1e6:9.1f}")
    print(f"batch total: read {tot_r / 1e9:.2f} GB, write {tot_w / 1e9:.2f} GB, sum {(tot_r + tot_w) / 1e9:.2f} GB")


if __name__ == "__main__":
    main()
