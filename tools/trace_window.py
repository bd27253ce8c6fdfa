"""Per-replay kernel mix from a ``rocprofv3 --kernel-trace`` CSV, restricted to the steady
state: the window between the ``--skip``-th and the last launch of a marker kernel (one per
replay, e.g. the fused softmax + top-k at the end of every CNN plan), so compile-time
launches (weight uploads, fp8 calibration, warm-up) are excluded.

    python tools/trace_window.py gpurun_out/prof/run_kernel_trace.csv --marker softmax_topk --skip 3

Prints, per kernel name, launches per replay and the share of kernel time in the window.
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="softmax_topk")
    ap.add_argument("--skip", type=int, default=3, help="replays at the start to leave out")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    name_key = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r[name_key]]
    if len(marks) <= a.skip + 1:
        raise SystemExit(f"only {len(marks)} launches of {a.marker!r}")
    lo, hi = marks[a.skip], marks[-1]
    replays = len(marks) - 1 - a.skip
    calls = collections.Counter()
    dur = collections.Counter()
    for r in rows[lo + 1:hi + 1]:
        n = r[name_key]
        calls[n] += 1
        dur[n] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(dur.values())
    t0, t1 = int(rows[lo]["End_Timestamp"]), int(rows[hi]["End_Timestamp"])
    print(f"window: {replays} replays, {(t1 - t0) / 1e6:.2f} ms wall, {tot / 1e6:.2f} ms kernel time "
          f"({tot / max(1, replays) / 1e3:.1f} us per replay)")
    for n, d in dur.most_common(a.top):
        print(f"{100 * d / tot:5.1f}%  {calls[n] / replays:6.2f}/replay  {d / calls[n] / 1e3:8.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
