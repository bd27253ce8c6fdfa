"""Per-dispatch view of one plan replay from a rocprofv3 kernel trace: lists the kernels
of the last complete replay (between two occurrences of a marker kernel) with durations,
grid sizes and short names.  usage: trace_layers.py TRACE.csv [MARKER_SUBSTRING]"""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
    return (m.group(1) if m else name)[:70]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "preprocess_kernel"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(idx) < 2:
        sys.exit("marker kernel not found twice")
    a, b = idx[-2], idx[-1]
    seg = rows[a:b]
    tot = 0.0
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        print(f"{d:9.1f}us wg={wg:7d} vgpr={r['VGPR_Count']:>4} {short(r['Kernel_Name'])}")
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    print(f"sum {tot:.1f}us  span {span:.1f}us  kernels {len(seg)}")


if __name__ == "__main__":
    main()
