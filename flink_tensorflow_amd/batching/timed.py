"""A timed window inside a streaming job: the benchmark contract (W untimed warm-up
micro-batches, then exactly K timed ones bracketed by a barrier + device synchronize on
both sides, elapsed = max over ranks) measured on the operator itself, so ``bench.py
--job`` can time the real job shape — one DataStream job whose P worker-process subtasks
each own a GPU, the source chained into them, the weights read once and broadcast over the
operator's communicator — instead of P independent SPMD pipelines.

``TimedWindow`` is a mixin for a ``BatchedGpuModel`` (``submit`` / ``poll`` / ``drain``):
it counts ``submit`` calls (one per micro-batch), fences before the first timed batch and
after the last one (drain the pipeline, synchronize, barrier on the operator's
communicator, synchronize), keeps the per-record latencies of the timed batches and writes
``{rank, elapsed_s, records, latencies}`` to ``<out_dir>/rank<r>.json`` at the second fence.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np


class TimedWindow:
    def timed_window(self, warmup: int, steps: int, out_dir: str):
        self._tw = {"w": int(warmup), "k": int(steps), "dir": out_dir, "n": 0, "t0": None, "lat": [],
                    "records": 0}
        return self

    def _fence(self) -> list:
        import torch

        from ..parallel import comm

        done = super().drain()
        dev = torch.cuda.current_device() if torch.cuda.is_available() else None
        if dev is not None:
            torch.cuda.synchronize(dev)
        comm.barrier()
        if dev is not None:
            torch.cuda.synchronize(dev)
        return done

    def _keep(self, results: list) -> list:
        tw = self._tw
        if tw["t0"] is not None:
            for _, _, lat in results:
                tw["lat"].append(np.asarray(lat, np.float64).reshape(-1))
        return results

    def submit(self, records, ingest_ts, tags):
        tw = self._tw
        i = tw["n"]
        tw["n"] += 1
        out = []
        if i == tw["w"]:
            out += self._fence()  # warm-up results: not timed
            tw["t0"] = time.perf_counter()
            tw["host0"] = self._host_s()
        if tw["w"] <= i < tw["w"] + tw["k"]:
            tw["records"] += len(records)
        out += self._keep(super().submit(records, ingest_ts, tags))
        if i == tw["w"] + tw["k"] - 1:
            out += self._keep(self._fence())
            elapsed = time.perf_counter() - tw["t0"]
            self._write(elapsed)
            tw["t0"] = None
        return out

    def poll(self):
        return self._keep(super().poll())

    def _host_s(self) -> dict:
        """The GPU runner's cumulative host seconds per phase (gather / decode, select,
        launch, wait), when the model has one."""
        r = getattr(self, "_runner", None)
        return dict(getattr(r, "host_s", {}) or {})

    def _write(self, elapsed: float) -> None:
        from ..parallel import comm

        tw = self._tw
        rank = comm.rank_size()[0]
        lat = np.concatenate(tw["lat"]) if tw["lat"] else np.zeros(0)
        os.makedirs(tw["dir"], exist_ok=True)
        tmp = os.path.join(tw["dir"], f".rank{rank}.json")
        with open(tmp, "w") as f:
            h0, h1 = tw.get("host0") or {}, self._host_s()
            host = {k: round((v - h0.get(k, 0.0)) * 1e3 / max(1, tw["k"]), 3) for k, v in h1.items()}
            ps = getattr(self, "plan_summary", None)
            try:
                plan = ps() if callable(ps) else None
            except Exception:  # noqa: BLE001  (diagnostics only)
                plan = None
            json.dump({"rank": rank, "world": comm.rank_size()[1], "elapsed_s": elapsed, "records": tw["records"],
                       "latencies_s": lat.tolist(), "pid": os.getpid(), "host_ms_per_batch": host, "plan": plan,
                       "communicator": type(comm.get()).__name__ if comm.is_dist() else None}, f, default=str)
        os.replace(tmp, os.path.join(tw["dir"], f"rank{rank}.json"))


class TimedSteps:
    """The same contract for a step-driven operator (``runtime/lockstep.py``
    ``LockstepTrainer``: agreed training steps, so every rank reaches step ``W`` and step
    ``W + K`` in the same round): fence after the ``W``-th step, count the records of the
    next ``K`` steps, fence after step ``W + K`` and write ``rank<r>.json``."""

    def timed_window(self, warmup: int, steps: int, out_dir: str):
        self._tw = {"w": int(warmup), "k": int(steps), "dir": out_dir, "t0": None, "records": 0}
        return self

    def _fence(self) -> None:
        import torch

        from ..parallel import comm

        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if comm.is_dist():
            comm.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def on_step(self, plan, piece, loss, out, counts=None):
        from ..runtime.lockstep import piece_len

        tw = self._tw
        i = self.steps  # steps done, this one included
        if tw["t0"] is not None:
            tw["records"] += piece_len(piece)
        if i == tw["w"]:
            self._fence()
            tw["t0"] = time.perf_counter()
        elif i == tw["w"] + tw["k"] and tw["t0"] is not None:
            self._fence()
            self._write_steps(time.perf_counter() - tw["t0"])
            tw["t0"] = None

    def _write_steps(self, elapsed: float) -> None:
        from ..parallel import comm

        tw = self._tw
        rank, world = comm.rank_size()
        os.makedirs(tw["dir"], exist_ok=True)
        tmp = os.path.join(tw["dir"], f".rank{rank}.json")
        with open(tmp, "w") as f:
            json.dump({"rank": rank, "world": world, "elapsed_s": elapsed, "records": tw["records"],
                       "steps": tw["k"], "rounds": getattr(self, "rounds", None)}, f)
        os.replace(tmp, os.path.join(tw["dir"], f"rank{rank}.json"))
