"""Concurrency of a multi-lane run from a rocprofv3 rocpd database: per timed window, the
sum of kernel durations, the union of kernel intervals (GPU busy) and the wall time, so
the lane overlap (sum / busy) and the idle fraction (1 - busy / wall) can be read off.
usage: lane_overlap.py results.db [n_batches=20] [marker=preprocess]"""
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    marker = sys.argv[3] if len(sys.argv) > 3 else "preprocess"
    rows = db.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    starts = [i for i, r in enumerate(rows) if marker in r[0]]
    if len(starts) < n:
        raise SystemExit(f"only {len(starts)} batches")
    first = starts[-n]
    win = rows[first:]
    t0, t1 = win[0][1], max(r[2] for r in win)
    tot = sum(r[2] - r[1] for r in win)
    busy, cur_s, cur_e = 0, None, None
    for _, s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = t1 - t0
    print(f"last {n} batches: wall {wall / 1e3:.0f} us ({wall / n / 1e3:.0f} us/batch), kernel sum "
          f"{tot / 1e3:.0f} us ({tot / n / 1e3:.0f} us/batch), busy {busy / 1e3:.0f} us; overlap sum/busy "
          f"{tot / busy:.2f}, idle {100 * (1 - busy / wall):.1f} %")
    # idle gaps > 20 us
    gaps, cur = [], win[0][2]
    for r in win[1:]:
        if r[1] > cur + 20000:
            gaps.append(((r[1] - cur) / 1e3, r[0][:60]))
        cur = max(cur, r[2])
    print(f"{len(gaps)} idle gaps > 20 us, total {sum(g[0] for g in gaps):.0f} us; largest:",
          sorted(gaps, reverse=True)[:5])


if __name__ == "__main__":
    main()
