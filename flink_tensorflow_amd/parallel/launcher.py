"""Supervised one-process-per-GPU launcher with failure detection and restarts
(SURVEY §5.3).

The reference delegates failure handling to Flink's restart strategies.  Here the driver
process spawns one worker per rank, each creating the job's RCCL communicator on its GPU
(``comm.init_distributed``; CPU tests inject the loopback ``parallel.fake`` communicator),
and supervises them:

* **exit detection** — a worker that dies (HIP error → non-zero exit, abort, kill) fails
  the attempt;
* **hang detection** — workers call :func:`heartbeat` from their step loop; a rank whose
  last beat is older than ``heartbeat_timeout`` fails the attempt (a wedged collective or
  kernel never returns to Python, so progress beats are the signal);
* **restart** — the whole group is torn down (the surviving ranks are killed by PID: a
  collective communicator cannot lose a member) and relaunched with ``attempt + 1`` on a
  fresh rendezvous port, up to ``max_restarts`` times; a worker that fails aborts its RCCL
communicator (no waiting on dead peers).  The worker function receives the
  attempt number and resumes from its latest checkpoint (e.g. a streaming job with
  ``restore_from_latest``); the communicator is re-created by the new processes.

``launch`` returns the per-rank return values of the successful attempt.
"""
from __future__ import annotations

import os
import queue
import socket
import time
import traceback
from dataclasses import dataclass, field
from typing import Any, Callable

import torch.multiprocessing as mp

_BEAT_Q = None
_RANK = 0


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def heartbeat(note: str = "") -> None:
    """Progress beat from inside a worker (no-op outside a launched worker)."""
    if _BEAT_Q is not None:
        try:
            _BEAT_Q.put_nowait(("beat", _RANK, time.time(), note))
        except Exception:  # noqa: BLE001
            pass


def _worker(rank: int, world: int, port: int, attempt: int, communicator, fn, args, q, env):
    global _BEAT_Q, _RANK
    _BEAT_Q, _RANK = q, rank
    os.environ.update(env)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), FTM_ATTEMPT=str(attempt))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from . import comm

    try:
        comm.init_distributed(communicator=communicator)
        heartbeat("init")
        res = fn(rank, world, attempt, *args)
        q.put(("done", rank, time.time(), res))
        comm.destroy()
    except BaseException as e:  # noqa: BLE001
        q.put(("error", rank, time.time(), f"{type(e).__name__}: {e}\n{traceback.format_exc()}"))
        comm.destroy(abort=True)
        raise SystemExit(1)


class WorkerFailure(RuntimeError):
    pass


@dataclass
class LaunchReport:
    results: list
    attempts: int
    failures: list = field(default_factory=list)


def launch(fn: Callable[..., Any], nprocs: int, args: tuple = (), communicator: type | None = None,
           max_restarts: int = 0, heartbeat_timeout: float | None = None, timeout: float | None = None,
           env: dict | None = None, restart_delay_s: float = 0.0) -> LaunchReport:
    """Runs ``fn(rank, world, attempt, *args)`` in ``nprocs`` supervised processes.
    ``communicator`` (a picklable ``comm.Communicator`` class) replaces RCCL — tests only."""
    ctx = mp.get_context("spawn")
    failures = []
    for attempt in range(max_restarts + 1):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, nprocs, port, attempt, communicator, fn, args, q, env or {}),
                             daemon=False) for r in range(nprocs)]
        for p in procs:
            p.start()
        start = time.time()
        last = {r: start for r in range(nprocs)}
        results: dict[int, Any] = {}
        reason = None
        while reason is None and len(results) < nprocs:
            try:
                kind, rank, ts, payload = q.get(timeout=0.2)
                last[rank] = time.time()
                if kind == "done":
                    results[rank] = payload
                elif kind == "error":
                    reason = f"rank {rank} raised: {payload}"
            except queue.Empty:
                pass
            now = time.time()
            exited = [r for r, p in enumerate(procs) if r not in results and p.exitcode is not None]
            if exited and reason is None:
                # a rank may have posted 'done' just before exiting: drain once more, then any
                # exited rank without a result failed — whatever its exit code (sys.exit(0)
                # inside fn, os._exit) — or the attempt would wait forever
                try:
                    while True:
                        kind, rank, ts, payload = q.get(timeout=0.05)
                        if kind == "done":
                            results[rank] = payload
                        elif kind == "error":
                            reason = f"rank {rank} raised: {payload}"
                except queue.Empty:
                    pass
                for r in exited:
                    if r not in results:
                        reason = reason or f"rank {r} exited with code {procs[r].exitcode} without a result"
            if heartbeat_timeout is not None:
                stale = [r for r in range(nprocs) if r not in results and now - last[r] > heartbeat_timeout]
                if stale:
                    reason = reason or f"ranks {stale} missed heartbeats for {heartbeat_timeout}s (hung)"
            if timeout is not None and now - start > timeout:
                reason = reason or f"attempt exceeded {timeout}s"
        if reason is None:
            for p in procs:
                p.join(timeout=30)
            return LaunchReport([results[r] for r in range(nprocs)], attempt + 1, failures)
        failures.append(reason)
        for p in procs:  # tear the group down: kill our own workers by PID
            if p.is_alive():
                p.kill()
        for p in procs:
            p.join(timeout=30)
        if attempt < max_restarts and restart_delay_s:
            time.sleep(restart_delay_s)
    raise WorkerFailure(f"job failed after {max_restarts + 1} attempt(s): " + " | ".join(failures))
