"""Operator metrics: counters, meters and latency histograms.

The reference has no metrics at all (no metric group, counters or histograms).  Every
subtask here gets a ``MetricGroup`` with ``records_in/out``, a batch-size histogram and a
per-record latency histogram (ingest → result) that yields p50/p95/p99; the driver
aggregates them (``all_gather`` in distributed mode) and exports JSON lines.
"""
from __future__ import annotations

import json
import threading
import time

import numpy as np


class Histogram:
    """Reservoir-free histogram keeping raw samples up to a cap, then decimating."""

    def __init__(self, cap: int = 200_000):
        self.cap = cap
        self._v: list[float] = []
        self.count = 0
        self._lock = threading.Lock()

    def update(self, v: float):
        with self._lock:
            self.count += 1
            self._v.append(float(v))
            if len(self._v) > self.cap:
                self._v = self._v[::2]

    def update_many(self, vs):
        with self._lock:
            vs = np.asarray(vs, dtype=np.float64).reshape(-1)
            self.count += len(vs)
            self._v.extend(vs.tolist())
            if len(self._v) > self.cap:
                self._v = self._v[:: max(2, len(self._v) // self.cap)]

    def percentile(self, q: float) -> float:
        with self._lock:
            return float(np.percentile(self._v, q)) if self._v else float("nan")

    def snapshot(self) -> dict:
        with self._lock:
            if not self._v:
                return {"count": self.count}
            a = np.asarray(self._v)
        return {"count": self.count, "mean": float(a.mean()), "p50": float(np.percentile(a, 50)),
                "p95": float(np.percentile(a, 95)), "p99": float(np.percentile(a, 99)), "max": float(a.max())}


class MetricGroup:
    def __init__(self, name: str):
        self.name = name
        self.counters: dict[str, int] = {}
        self.histograms: dict[str, Histogram] = {}
        self.gauges: dict[str, float] = {}
        self.t0 = time.time()
        self._lock = threading.Lock()

    def inc(self, name: str, n: int = 1):
        with self._lock:
            self.counters[name] = self.counters.get(name, 0) + n

    def counter(self, name: str) -> int:
        return self.counters.get(name, 0)

    def histogram(self, name: str) -> Histogram:
        with self._lock:
            h = self.histograms.get(name)
            if h is None:
                h = self.histograms[name] = Histogram()
            return h

    def gauge(self, name: str, value: float):
        self.gauges[name] = float(value)

    def snapshot(self) -> dict:
        el = max(time.time() - self.t0, 1e-9)
        out = {"counters": dict(self.counters), "gauges": dict(self.gauges),
               "rates": {k + "_per_s": v / el for k, v in self.counters.items()},
               "histograms": {k: h.snapshot() for k, h in self.histograms.items()}}
        return out

    def to_json(self) -> str:
        return json.dumps({"name": self.name, **self.snapshot()})


class BucketHistogram:
    """Log-spaced fixed buckets (0.5 % relative width, 1e-7 .. 1e4): mergeable by summing counts.

    Percentiles of a merged ``BucketHistogram`` are whole-job percentiles (not a median of
    per-rank percentiles): ``parallel.comm.allgather_metrics`` sums the count vectors of all
    ranks with one all-reduce of a fixed-size int64 tensor.
    """
    LO = 1e-7
    GROWTH = 1.005
    N = int(np.ceil(np.log(1e4 / 1e-7) / np.log(1.005))) + 1

    def __init__(self, counts=None):
        self.counts = np.zeros(self.N, np.int64) if counts is None else np.asarray(counts, np.int64).copy()

    @classmethod
    def index(cls, vs) -> np.ndarray:
        v = np.maximum(np.asarray(vs, np.float64).reshape(-1), cls.LO)
        return np.minimum((np.log(v / cls.LO) / np.log(cls.GROWTH)).astype(np.int64), cls.N - 1)

    def update_many(self, vs):
        np.add.at(self.counts, self.index(vs), 1)

    def merge(self, other: "BucketHistogram") -> "BucketHistogram":
        self.counts += other.counts
        return self

    @property
    def count(self) -> int:
        return int(self.counts.sum())

    def percentile(self, q: float) -> float:
        n = self.count
        if n == 0:
            return float("nan")
        rank = min(n - 1, max(0, int(np.ceil(q / 100.0 * n)) - 1))
        i = int(np.searchsorted(np.cumsum(self.counts), rank + 1))
        return float(self.LO * self.GROWTH ** (i + 0.5))     # bucket's geometric midpoint

    def snapshot(self) -> dict:
        if self.count == 0:
            return {"count": 0}
        return {"count": self.count, "p50": self.percentile(50), "p95": self.percentile(95),
                "p99": self.percentile(99), "max": self.percentile(100)}


def histogram_buckets(h: Histogram) -> BucketHistogram:
    """Bins a raw-sample ``Histogram`` (decimated samples are re-weighted to ``h.count``)."""
    with h._lock:
        v = np.asarray(h._v, np.float64)
        count = h.count
    b = BucketHistogram()
    if len(v):
        b.update_many(v)
        if count != len(v):          # decimated: scale counts back to the true total
            b.counts = np.round(b.counts * (count / len(v))).astype(np.int64)
    return b
