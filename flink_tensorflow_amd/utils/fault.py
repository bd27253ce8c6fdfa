"""Fault injection for recovery tests: fail a subtask after N records on
chosen attempts, or corrupt a checkpoint file (caught by the CRC32C bundle checks)."""
from __future__ import annotations

import os

from ..runtime.functions import RichMapFunction


class InjectedFault(RuntimeError):
    pass


class FailAfter(RichMapFunction):
    """Identity map that raises on the ``n``-th record of subtask ``subtask`` during the
    listed restart ``attempts`` (attempt 0 = first run)."""

    def __init__(self, n: int, attempts=(0,), subtask: int = 0):
        super().__init__()
        self.n, self.attempts, self.subtask = n, tuple(attempts), subtask
        self.seen = 0

    def map(self, value):
        ctx = self.get_runtime_context()
        self.seen += 1
        if ctx.attempt in self.attempts and ctx.subtask_index == self.subtask and self.seen == self.n:
            raise InjectedFault(f"injected failure at record {self.n} (attempt {ctx.attempt})")
        return value


class KillProcessAfter(FailAfter):
    """Like ``FailAfter`` but the subtask's PROCESS dies (``os._exit``, no Python unwinding,
    no goodbye message) — a crashed worker of ``run_in_processes()``: the coordinator must
    detect the dead process and restart the job from the last completed checkpoint."""

    def __init__(self, n: int, attempts=(0,), subtask: int = 0, exit_code: int = 137):
        super().__init__(n, attempts, subtask)
        self.exit_code = exit_code

    def map(self, value):
        ctx = self.get_runtime_context()
        self.seen += 1
        if ctx.attempt in self.attempts and ctx.subtask_index == self.subtask and self.seen == self.n:
            if getattr(ctx, "worker_pid", None) != os.getpid():
                raise InjectedFault("KillProcessAfter must run in a worker process (run_in_processes)")
            os._exit(self.exit_code)
        return value


class FaultInjector:
    """Hook object for ``env.fault_injector`` (armed at each job attempt)."""

    def __init__(self):
        self.armed_attempts: list[int] = []

    def arm(self, executor):
        self.armed_attempts.append(executor.attempt)

    @staticmethod
    def corrupt_file(path: str, offset: int = 0):
        with open(path, "r+b") as f:
            f.seek(offset)
            b = f.read(1)
            f.seek(offset)
            f.write(bytes([b[0] ^ 0xFF]) if b else b"\xff")
        return os.path.getsize(path)
