"""Per-forward breakdown of a rocprofv3 kernel trace (csv): the last forward of the run,
one line per dispatch, plus a per-kernel-name summary."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
marker = sys.argv[2] if len(sys.argv) > 2 else "preprocess"
rows = list(csv.DictReader(open(path)))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
s = idx[-1]
e = len(rows)
tot = 0.0
agg = defaultdict(float)
for r in rows[s:e]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += d
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")
    agg[name] += d
    if "-v" in sys.argv:
        print(f"{d:8.1f}us grid={int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):7d} lds={r['LDS_Block_Size']:>6} "
              f"vgpr={r['VGPR_Count']:>4} {name[:90]}")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]):
    print(f"{v:9.1f}us {100*v/tot:5.1f}%  {k[:100]}")
print(f"total {tot:.1f}us")
