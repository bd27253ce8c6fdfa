"""Batch-by-batch account of bench.py's timed window: reads the
``{"timeline": [...], "elapsed_ms": ...}`` line ``bench.py --timeline`` prints (per batch:
lane, host submit, first H2D done, first kernel start, compute done; ms from the window's
start) and splits the window into startup (before the first kernel), steady state (the
median per-batch period over both lanes, from consecutive completions) and the tail after
the last full period.  usage: window_timeline.py bench_timeline.log [...]"""
import json
import sys


def analyse(tl: list, elapsed: float) -> dict:
    tl = sorted(tl, key=lambda b: b["done_ms"])
    done = [b["done_ms"] for b in tl]
    # steady per-batch period over both lanes: completions alternate lanes, so take the
    # slope between the 3rd and the 3rd-last completion (no fill, no drain)
    k = min(2, max(0, (len(done) - 2) // 2))
    period = (done[-1 - k] - done[k]) / max(1, len(done) - 1 - 2 * k)
    first_start = min(b["start_ms"] for b in tl)
    first_done = done[0]
    n = len(tl)
    ideal = n * period
    lanes = sorted({b["lane"] for b in tl})
    last_by_lane = {ln: max(b["done_ms"] for b in tl if b["lane"] == ln) for ln in lanes}
    return {"batches": n, "elapsed_ms": round(elapsed, 3), "period_ms": round(period, 3),
            "ideal_ms": round(ideal, 3), "overhead_ms": round(elapsed - ideal, 3),
            "overhead_pct": round(100 * (elapsed - ideal) / elapsed, 2),
            "first_submit_ms": round(min(b["submit_ms"] for b in tl), 3),
            "first_kernel_ms": round(first_start, 3), "first_done_ms": round(first_done, 3),
            "lane_finish_spread_ms": round(max(last_by_lane.values()) - min(last_by_lane.values()), 3),
            "last_done_ms": round(done[-1], 3)}


def main():
    for path in sys.argv[1:]:
        for line in open(path):
            if line.startswith('{"timeline"'):
                d = json.loads(line)
                print(json.dumps({"file": path, **analyse(d["timeline"], d["elapsed_ms"])}))


if __name__ == "__main__":
    main()
