#!/usr/bin/env python3
"""Host side of an 8-rank node, without the GPUs.

Each DP rank of the headline job stages one 256-image micro-batch (256 x 196,608 B of
decoded uint8 records, 50.3 MB) into a host slot per step with the native multithreaded
gather (``csrc/native.cpp`` ``gather_into``, what ``batching/engine.py``'s runner calls),
and the GPU then DMA-reads that slot.  This tool starts R such stagers as separate
processes, each bound to the NUMA node its GPU would have (the ``numa_node`` of the R-th
AMD GPU PCI function in sysfs, round-robin over the host's nodes when there are fewer),
first-touching its pool and slots there, and runs them concurrently for ``--seconds``:

* per rank: gather ms per micro-batch (p50 / p99) against the step budget
  (``--step-ms``, default 3.3 ms = 77.5k images/s per GPU);
* aggregate: GB/s written into the slots by all ranks together, and what R ranks at the
  per-GPU target rate need (``R x 50.3 MB / step``).

No GPU is touched (no HIP call, no torch.cuda): slots are plain 2 MiB-aligned host memory
(the pinned slots of a real run are the same pages plus the DMA reads, which this does not
generate — reported as the remaining headroom).  Prints one JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REC = 256 * 256 * 3


def _cpulist(text: str) -> set[int]:
    out: set[int] = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def gpu_numa_nodes() -> list[int]:
    """numa_node of every AMD GPU / accelerator PCI function (vendor 0x1002, display or
    processing-accelerator class), in PCI order."""
    nodes = []
    for d in sorted(glob.glob("/sys/bus/pci/devices/*")):
        try:
            vendor = open(os.path.join(d, "vendor")).read().strip()
            cls = open(os.path.join(d, "class")).read().strip()
            if vendor != "0x1002" or not (cls.startswith("0x0380") or cls.startswith("0x0300")
                                          or cls.startswith("0x1200")):
                continue
            nodes.append(int(open(os.path.join(d, "numa_node")).read()))
        except (OSError, ValueError):
            continue
    return nodes


def host_nodes() -> dict[int, set[int]]:
    out = {}
    for d in glob.glob("/sys/devices/system/node/node[0-9]*"):
        try:
            out[int(d.rsplit("node", 1)[1])] = _cpulist(open(os.path.join(d, "cpulist")).read())
        except (OSError, ValueError):
            pass
    return out


def _rank(r: int, node: int | None, cpus: list[int], args, start, q) -> None:
    from flink_tensorflow_amd import _ext

    if cpus:
        os.sched_setaffinity(0, cpus)  # the gather pool's threads inherit the mask
    nat = _ext.native()
    rng = np.random.default_rng(100 + r)
    pool = rng.integers(0, 256, size=(args.pool, REC), dtype=np.uint8)  # first-touched on this node
    recs = [pool[i] for i in range(args.pool)]
    B = args.batch
    slots = []
    for _ in range(args.depth):
        raw = np.empty(B * REC + (2 << 20), np.uint8)
        off = (-raw.ctypes.data) % (2 << 20)
        s = raw[off:off + B * REC]
        s.fill(0)  # first touch
        slots.append(s)
    batch = [recs[i % args.pool] for i in range(B)]
    for i in range(3):  # warm-up
        nat.gather_into(slots[i % args.depth].ctypes.data, B * REC, batch, REC, args.threads)
    start.wait()
    times = []
    t_end = time.perf_counter() + args.seconds
    k = 0
    while time.perf_counter() < t_end:
        batch = [recs[(k * B + i) % args.pool] for i in range(B)]
        t0 = time.perf_counter()
        nat.gather_into(slots[k % args.depth].ctypes.data, B * REC, batch, REC, args.threads)
        times.append(time.perf_counter() - t0)
        k += 1
        if args.paced:  # a real rank stages once per step: sleep out the rest of it
            rest = args.step_ms / 1e3 - times[-1]
            if rest > 0:
                time.sleep(rest)
    q.put({"rank": r, "numa_node": node, "cpus": len(cpus), "batches": k, "bytes": k * B * REC,
           "busy_s": float(np.sum(times)), "p50_ms": float(np.percentile(times, 50) * 1e3),
           "p99_ms": float(np.percentile(times, 99) * 1e3)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=2, help="gather threads per rank")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--pool", type=int, default=96, help="distinct records per rank (96 x 196 KB = 18.9 MB)")
    ap.add_argument("--depth", type=int, default=3, help="host slots per rank")
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--step-ms", type=float, default=3.3)
    ap.add_argument("--paced", action="store_true", help="one gather per --step-ms per rank (the real duty cycle)")
    args = ap.parse_args()

    gnodes = gpu_numa_nodes()
    hnodes = host_nodes()
    allowed = os.sched_getaffinity(0)
    node_ids = sorted(hnodes) or [None]
    plan = []
    for r in range(args.ranks):
        node = gnodes[r] if r < len(gnodes) and gnodes[r] >= 0 else node_ids[r * len(node_ids) // args.ranks]
        cpus = sorted(hnodes.get(node, allowed) & allowed) if node is not None else sorted(allowed)
        plan.append((node, cpus))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    start = ctx.Event()
    procs = [ctx.Process(target=_rank, args=(r, n, c, args, start, q)) for r, (n, c) in enumerate(plan)]
    for p in procs:
        p.start()
    time.sleep(2.0)
    t0 = time.perf_counter()
    start.set()
    res = [q.get(timeout=args.seconds + 120) for _ in procs]
    for p in procs:
        p.join(30)
    wall = time.perf_counter() - t0
    res.sort(key=lambda x: x["rank"])
    total = sum(x["bytes"] for x in res)
    need = args.ranks * args.batch * REC / (args.step_ms / 1e3)
    print(json.dumps({
        "tool": "host_staging_rehearsal", "ranks": args.ranks, "threads_per_rank": args.threads,
        "paced": args.paced, "batch": args.batch, "record_bytes": REC, "allowed_cpus": len(allowed),
        "gpu_numa_nodes_sysfs": gnodes, "host_numa_nodes": {k: len(v) for k, v in hnodes.items()},
        "aggregate_gather_GBps": round(total / wall / 1e9, 1),
        "needed_GBps_at_step": round(need / 1e9, 1), "step_ms": args.step_ms,
        "per_rank": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in x.items()} for x in res],
        "worst_p99_ms": round(max(x["p99_ms"] for x in res), 3),
        "worst_p50_ms": round(max(x["p50_ms"] for x in res), 3)}), flush=True)


if __name__ == "__main__":
    main()
