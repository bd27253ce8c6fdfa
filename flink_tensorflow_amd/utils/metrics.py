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
