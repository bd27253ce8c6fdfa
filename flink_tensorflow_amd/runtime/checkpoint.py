"""Checkpoint coordinator, storage and restart strategies.

Chandy-Lamport aligned barriers: the coordinator triggers checkpoint ``n`` at sources,
which emit ``Barrier(n)`` between records while holding their checkpoint lock (source
offsets are part of the snapshot).  Every task aligns barriers over its input channels,
flushes in-flight micro-batches, snapshots operator/keyed/model state, acknowledges and
forwards the barrier.  When all tasks acknowledged, the checkpoint is written:

    <dir>/chk-<n>/<task-uid>-<subtask>.state     pickled operator state (our own files)
    <dir>/chk-<n>/models/...                       CheckpointedModel bundles (TensorBundle V2)
    <dir>/chk-<n>/_metadata.json                   manifest (written last = commit point)

On failure the executor restarts the job from the latest committed checkpoint according
to the restart strategy (fixed delay, N attempts), and sources rewind to their offsets.
"""
from __future__ import annotations

import json
import os
import pickle
import shutil
import threading
import time
from dataclasses import dataclass


@dataclass
class RestartStrategy:
    attempts: int = 0
    delay_s: float = 0.0

    @staticmethod
    def no_restart() -> "RestartStrategy":
        return RestartStrategy(0, 0.0)

    @staticmethod
    def fixed_delay(attempts: int, delay_s: float = 0.0) -> "RestartStrategy":
        return RestartStrategy(attempts, delay_s)


class CheckpointStorage:
    def __init__(self, root: str, retain: int = 3):
        self.root = root
        self.retain = retain
        os.makedirs(root, exist_ok=True)

    def chk_dir(self, cid: int) -> str:
        return os.path.join(self.root, f"chk-{cid}")

    def write(self, cid: int, states: dict[tuple[str, int], dict], meta: dict) -> str:
        d = self.chk_dir(cid)
        os.makedirs(d, exist_ok=True)
        files = {}
        for (uid, sub), st in states.items():
            fn = f"{uid}-{sub}.state"
            with open(os.path.join(d, fn), "wb") as f:
                pickle.dump(st, f, protocol=pickle.HIGHEST_PROTOCOL)
            files[f"{uid}/{sub}"] = fn
        manifest = {"checkpoint_id": cid, "timestamp": time.time(), "files": files, **meta}
        tmp = os.path.join(d, "_metadata.json.tmp")
        with open(tmp, "w") as f:
            json.dump(manifest, f)
        os.replace(tmp, os.path.join(d, "_metadata.json"))
        self._gc()
        return d

    def _gc(self):
        done = self.completed()
        for cid in done[:-self.retain] if self.retain else []:
            shutil.rmtree(self.chk_dir(cid), ignore_errors=True)

    def completed(self) -> list[int]:
        out = []
        for n in os.listdir(self.root):
            if n.startswith("chk-") and os.path.exists(os.path.join(self.root, n, "_metadata.json")):
                out.append(int(n[4:]))
        return sorted(out)

    def latest(self) -> int | None:
        c = self.completed()
        return c[-1] if c else None

    def load(self, cid: int) -> dict[tuple[str, int], dict]:
        d = self.chk_dir(cid)
        with open(os.path.join(d, "_metadata.json")) as f:
            manifest = json.load(f)
        out = {}
        for key, fn in manifest["files"].items():
            uid, sub = key.rsplit("/", 1)
            with open(os.path.join(d, fn), "rb") as f:  # files written by this module
                out[(uid, int(sub))] = pickle.load(f)
        return out


class CheckpointCoordinator:
    def __init__(self, storage: CheckpointStorage, interval_s: float, executor):
        self.storage = storage
        self.interval = interval_s
        self.executor = executor
        self.next_id = (storage.latest() or 0) + 1
        self.pending: dict[int, dict] = {}
        self.expected: set[tuple[str, int]] = set()
        self.lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.completed_ids: list[int] = []
        # state at end-of-input of tasks that finished (sources: their final offsets): part of
        # every later checkpoint, so a restore does not replay a finished source's records
        # into operators whose state already contains them
        self.final_states: dict[tuple[str, int], dict] = {}

    def start(self, expected_tasks: set[tuple[str, int]]):
        self.expected = set(expected_tasks)
        self.final_states = {}
        self._thread = threading.Thread(target=self._loop, name="checkpoint-coordinator", daemon=True)
        self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)

    def _loop(self):
        while not self._stop.wait(self.interval):
            self.trigger()

    def trigger(self) -> int | None:
        with self.lock:
            if self.pending:  # one checkpoint in flight at a time
                return None
            cid = self.next_id
            self.next_id += 1
            self.pending[cid] = {}
        self.executor.trigger_sources(cid)
        return cid

    def acknowledge(self, cid: int, task: tuple[str, int], state: dict):
        with self.lock:
            p = self.pending.get(cid)
            if p is None:
                return
            p[task] = state
            self._maybe_complete(cid)

    def task_finished(self, task: tuple[str, int], final_state: dict | None = None):
        with self.lock:
            self.expected.discard(task)
            if final_state is not None:
                self.final_states[task] = final_state
            for cid in list(self.pending):
                self._maybe_complete(cid)

    def _maybe_complete(self, cid):
        p = self.pending[cid]
        if self.expected and not self.expected.issubset(p.keys()):
            return
        del self.pending[cid]
        p = {**{t: st for t, st in self.final_states.items() if t not in p}, **p}
        self.storage.write(cid, p, {"tasks": sorted(f"{u}/{s}" for u, s in p)})
        self.completed_ids.append(cid)
        self.executor.notify_complete(cid)

    def abort_pending(self):
        with self.lock:
            self.pending.clear()
