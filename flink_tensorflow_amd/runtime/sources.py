"""Sources and sinks.

* ``CollectionSource`` — ``env.from_collection`` (checkpoints its offset; partitioned across
  subtasks and across ranks in distributed mode).
* ``env.read_file(format, path, PROCESS_ONCE | PROCESS_CONTINUOUSLY, interval)`` as Flink
  builds it: ``FileMonitorFunction`` (parallelism 1) lists the directory and forwards only
  the new files' PATHS, round-robin to the parallel
  ``FileReaderOperator`` subtasks, which read each file and run the format's
  ``read_record`` (decode, normalise) — chained into the worker process of the GPU
  operator they feed, so the coordinator ships a path per record, not the decoded tensor.
  Exactly one record per file (``LIB/io/WholeFileInputFormat.scala:14-80``); end
  detection is an explicit "emitted" flag, so zero-length files do not re-emit forever
  (B5); include/exclude glob filters are merged rather than overwritten (B8).
* ``FileMonitoringSource`` — the single-operator form (each subtask lists, reads and
  decodes the files hashed to it), for jobs that add it as a plain source.
* ``GeneratorSource`` — records from a Python generator factory (synthetic load).
* ``PrintSink``, ``MemorySink`` (``TST/.../util/MemorySinkFunction.java``), ``CollectSink``.
"""
from __future__ import annotations

import abc
import enum
import threading
import time
from collections import defaultdict
from typing import Any, Callable, Iterable, Sequence

from ..utils import fs
from .functions import CheckpointedFunction, SinkFunction, SourceFunction
from .state import ListStateDescriptor


class FileProcessingMode(enum.Enum):
    PROCESS_ONCE = 0
    PROCESS_CONTINUOUSLY = 1


PROCESS_ONCE = FileProcessingMode.PROCESS_ONCE
PROCESS_CONTINUOUSLY = FileProcessingMode.PROCESS_CONTINUOUSLY


def _partition(ctx):
    """(global subtask index, global parallelism) including the distributed rank."""
    return getattr(ctx, "global_index", ctx.subtask_index), getattr(ctx, "global_parallelism", ctx.parallelism)


class CollectionSource(SourceFunction, CheckpointedFunction):
    def __init__(self, items: Sequence, timestamps: Sequence[float] | None = None, delay_s: float = 0.0):
        super().__init__()
        self.items = list(items)
        self.timestamps = list(timestamps) if timestamps is not None else None
        self.delay = delay_s
        self.offset = 0
        self._running = True

    def initialize_state(self, ctx):
        self._state = ctx.operator_state.get_list_state(ListStateDescriptor("offset"))
        if ctx.is_restored():
            v = self._state.get()
            self.offset = v[0] if v else 0

    def snapshot_state(self, ctx):
        self._state.update([self.offset])

    def run(self, ctx):
        idx, par = _partition(self.get_runtime_context())
        mine = list(range(idx, len(self.items), par))
        while self.offset < len(mine) and self._running:
            with ctx.checkpoint_lock:
                i = mine[self.offset]
                ts = self.timestamps[i] if self.timestamps is not None else None
                ctx.collect(self.items[i], ts)
                self.offset += 1
            if self.delay:
                time.sleep(self.delay)

    def cancel(self):
        self._running = False


class GeneratorSource(SourceFunction, CheckpointedFunction):
    """Records from ``factory(subtask_index, parallelism, start_offset)`` (an iterator).

    Relocatable: a subtask's records depend only on its index, so the subtask can run in
    whichever process consumes them (``LocalExecutor._relocate_sources``)."""

    relocatable = True

    def __init__(self, factory: Callable[[int, int, int], Iterable], limit: int | None = None, bulk: bool = False):
        super().__init__()
        self.factory = factory
        self.limit = limit
        # bulk: the factory yields LISTS of records, each emitted as one run
        # (``SourceContext.collect_many``); offsets still count records
        self.bulk = bulk
        self.offset = 0
        self._running = True

    def initialize_state(self, ctx):
        self._state = ctx.operator_state.get_list_state(ListStateDescriptor("offset"))
        if ctx.is_restored():
            v = self._state.get()
            self.offset = v[0] if v else 0

    def snapshot_state(self, ctx):
        self._state.update([self.offset])

    def run(self, ctx):
        idx, par = _partition(self.get_runtime_context())
        for v in self.factory(idx, par, self.offset):
            if not self._running or (self.limit is not None and self.offset >= self.limit):
                break
            with ctx.checkpoint_lock:
                if self.bulk:
                    if self.limit is not None:
                        v = v[:self.limit - self.offset]
                    ctx.collect_many(v)
                    self.offset += len(v)
                else:
                    ctx.collect(v)
                    self.offset += 1

    def cancel(self):
        self._running = False


# ------------------------------------------------------------------ whole-file input
class WholeFileInputFormat(abc.ABC):
    """One record per file; unsplittable.  Subclasses implement ``read_record``."""

    def __init__(self, include: Sequence[str] | None = None, exclude: Sequence[str] | None = None):
        self.include = list(include or [])
        self.exclude = list(exclude or [])

    def configure(self, include: Sequence[str] = (), exclude: Sequence[str] = ()):
        """Adds filters (merged with the constructor's, not replacing them: B8)."""
        self.include += [p for p in include if p not in self.include]
        self.exclude += [p for p in exclude if p not in self.exclude]
        return self

    def open_input_format(self):  # noqa: B027  (source-owned models open here)
        pass

    def close_input_format(self):  # noqa: B027
        pass

    @abc.abstractmethod
    def read_record(self, path: str, data: bytes) -> Any:
        ...

    def files(self, root: str) -> list[str]:
        return fs.list_files(root, include=self.include or None, exclude=self.exclude or None)


class BytesInputFormat(WholeFileInputFormat):
    def read_record(self, path, data):
        return path, data


class FileMonitoringSource(SourceFunction, CheckpointedFunction):
    def __init__(self, fmt: WholeFileInputFormat, path: str, mode: FileProcessingMode = PROCESS_ONCE,
                 interval_s: float = 1.0, max_polls: int | None = None):
        super().__init__()
        self.fmt = fmt
        self.path = path
        self.mode = mode
        self.interval = interval_s
        self.max_polls = max_polls
        self.seen: set[str] = set()
        self._running = True

    def initialize_state(self, ctx):
        self._state = ctx.operator_state.get_list_state(ListStateDescriptor("seen"))
        if ctx.is_restored():
            self.seen = set(self._state.get())

    def snapshot_state(self, ctx):
        self._state.update(sorted(self.seen))

    def run(self, ctx):
        idx, par = _partition(self.get_runtime_context())
        self.fmt.open_input_format()
        try:
            polls = 0
            while self._running:
                files = [f for f in self.fmt.files(self.path) if f not in self.seen]
                for i, f in enumerate(sorted(files)):
                    if hash_str(f) % par != idx:
                        with ctx.checkpoint_lock:
                            self.seen.add(f)
                        continue
                    data = fs.read_bytes(f)
                    rec = self.fmt.read_record(f, data)
                    with ctx.checkpoint_lock:
                        if rec is not None:
                            ctx.collect(rec)
                        self.seen.add(f)  # emitted flag (B5): zero-length files emit once
                polls += 1
                if self.mode == PROCESS_ONCE or (self.max_polls is not None and polls >= self.max_polls):
                    break
                t_end = time.time() + self.interval
                while self._running and time.time() < t_end:
                    time.sleep(min(0.05, self.interval))
        finally:
            self.fmt.close_input_format()

    def cancel(self):
        self._running = False


class FileMonitorFunction(SourceFunction, CheckpointedFunction):
    """Flink's ``ContinuousFileMonitoringFunction``: lists ``path`` through the format's
    filters and emits each file not seen before as its path (a plain ``str``: a whole file
    is one split, and the path is all a reader needs) — nothing read or decoded here; PROCESS_CONTINUOUSLY re-lists every ``interval_s``.  Runs with
    parallelism 1; its checkpoint state is the set of paths already forwarded (a path
    forwarded before a barrier is read by its reader before the reader snapshots, so every
    file is read exactly once across restarts).  The format is never opened here (a
    source-owned model, ``ImageInputFormat``'s normaliser, loads in the readers)."""

    def __init__(self, fmt: WholeFileInputFormat, path: str, mode: FileProcessingMode = PROCESS_ONCE,
                 interval_s: float = 1.0, max_polls: int | None = None):
        super().__init__()
        self.fmt = fmt
        self.path = path
        self.mode = mode
        self.interval = interval_s
        self.max_polls = max_polls
        self.seen: set[str] = set()
        self._running = True

    def initialize_state(self, ctx):
        self._state = ctx.operator_state.get_list_state(ListStateDescriptor("seen"))
        if ctx.is_restored():
            self.seen = set(self._state.get())

    def snapshot_state(self, ctx):
        self._state.update(sorted(self.seen))

    def run(self, ctx):
        polls = 0
        while self._running:
            # oldest first, as Flink forwards splits by modification time
            for f in sorted((f for f in self.fmt.files(self.path) if f not in self.seen), key=_mtime_then_name):
                with ctx.checkpoint_lock:
                    ctx.collect(str(f))
                    self.seen.add(f)
            polls += 1
            if self.mode == PROCESS_ONCE or (self.max_polls is not None and polls >= self.max_polls):
                break
            t_end = time.time() + self.interval
            while self._running and time.time() < t_end:
                time.sleep(min(0.05, self.interval))

    def cancel(self):
        self._running = False


class PartitionedFileSource(SourceFunction, CheckpointedFunction):
    """``read_file(..., monitor="partitioned")``: the monitor and the reader in one source
    subtask per reader, each listing the directory itself and taking the files whose path
    hashes to its index (``crc32(path) % parallelism``), reading a run of them at once on the
    native host pool (``read_files``) and handing the run's records on as one run
    (``SourceContext.collect_many``).  Relocatable, so a subtask runs inside the worker
    process of the GPU operator it feeds: no path and no record crosses the coordinator,
    where the Flink-shaped monitor + readers (``FileMonitorFunction`` ->
    ``FileReaderOperator``) forward every path through it.  State: the paths already
    emitted by this subtask (as the monitor's), so a restore re-reads none of them."""

    relocatable = True

    def __init__(self, fmt: WholeFileInputFormat, path: str, mode: FileProcessingMode = PROCESS_ONCE,
                 interval_s: float = 1.0, max_polls: int | None = None, run: int = 64, read_threads: int = 8):
        super().__init__()
        self.fmt = fmt
        self.path = path
        self.mode = mode
        self.interval = interval_s
        self.max_polls = max_polls
        self.run_size = max(1, int(run))
        self.read_threads = read_threads
        self.seen: set[str] = set()
        self._running = True

    def initialize_state(self, ctx):
        self._state = ctx.operator_state.get_list_state(ListStateDescriptor("seen"))
        if ctx.is_restored():
            self.seen = set(self._state.get())

    def snapshot_state(self, ctx):
        self._state.update(sorted(self.seen))

    def open(self, parameters=None):
        self.fmt.open_input_format()

    def close(self):
        self.fmt.close_input_format()

    def _read(self, paths: list) -> list:
        blobs = [None] * len(paths)
        if isinstance(fs.get_fs(self.path)[0], fs.LocalFS):  # the listing's children are local too
            from .. import _ext

            blobs = _ext.native().read_files([fs.get_fs(p)[1] if "://" in p else p for p in paths],
                                             self.read_threads)
        # not local, or unreadable: the per-file path (raises with the OS error)
        return [b if b is not None else fs.read_bytes(p) for p, b in zip(paths, blobs)]

    def run(self, ctx):
        import zlib

        idx, par = _partition(self.get_runtime_context())
        polls = 0
        while self._running:
            mine = sorted((f for f in self.fmt.files(self.path)
                           if f not in self.seen and zlib.crc32(f.encode()) % par == idx), key=_mtime_then_name)
            for lo in range(0, len(mine), self.run_size):
                if not self._running:
                    return
                paths = mine[lo:lo + self.run_size]
                outs = [o for o in (self.fmt.read_record(p, d) for p, d in zip(paths, self._read(paths)))
                        if o is not None]
                with ctx.checkpoint_lock:
                    if outs:
                        ctx.collect_many(outs)
                    self.seen.update(paths)
            polls += 1
            if self.mode == PROCESS_ONCE or (self.max_polls is not None and polls >= self.max_polls):
                break
            t_end = time.time() + self.interval
            while self._running and time.time() < t_end:
                time.sleep(min(0.05, self.interval))

    def cancel(self):
        self._running = False


def _mtime_then_name(path: str):
    import os

    try:
        return (os.path.getmtime(path), path)
    except OSError:
        return (0.0, path)


def hash_str(s: str) -> int:
    import zlib

    return zlib.crc32(s.encode())


# ------------------------------------------------------------------ sinks
class PrintSink(SinkFunction):
    def __init__(self, prefix: str = "", stream=None):
        super().__init__()
        self.prefix = prefix
        self.stream = stream

    def invoke(self, value):
        ctx = self.get_runtime_context()
        tag = f"{ctx.subtask_index + 1}> " if ctx.parallelism > 1 else ""
        print(f"{self.prefix}{tag}{value}", file=self.stream, flush=True)


class MemorySink(SinkFunction):
    """Collects into a process-wide dict keyed by sink id (``MemorySinkFunction``)."""

    RESULTS: dict[int, list] = defaultdict(list)
    _LOCK = threading.Lock()
    _NEXT = [0]

    def __init__(self, key: int | None = None):
        super().__init__()
        with MemorySink._LOCK:
            if key is None:
                key = MemorySink._NEXT[0]
                MemorySink._NEXT[0] += 1
        self.key = key
        MemorySink.RESULTS.setdefault(key, [])

    def invoke(self, value):
        with MemorySink._LOCK:
            MemorySink.RESULTS[self.key].append(value)

    def results(self) -> list:
        with MemorySink._LOCK:
            return list(MemorySink.RESULTS[self.key])

    @classmethod
    def clear(cls, key: int | None = None):
        with cls._LOCK:
            if key is None:
                cls.RESULTS.clear()
            else:
                cls.RESULTS[key] = []


class CollectSink(MemorySink):
    """A MemorySink whose results are returned by ``DataStream.execute_and_collect``."""


class DiscardingSink(SinkFunction):
    """Flink's ``DiscardingSink``: drops every record (benchmarks; chained into a worker
    process, results never leave it)."""

    def invoke(self, value):
        pass


class ThroughputSink(SinkFunction):
    """Counts records and timestamps every ``every``-th one (process-wide registry keyed
    like ``MemorySink``): ``rate(skip_fraction)`` is the steady-state records/s after the
    warm-up part of the stream (compile, capture, pipeline fill)."""

    STAMPS: dict[int, list] = defaultdict(list)
    _LOCK = threading.Lock()
    _NEXT = [0]

    def __init__(self, every: int = 256):
        super().__init__()
        with ThroughputSink._LOCK:
            self.key = ThroughputSink._NEXT[0]
            ThroughputSink._NEXT[0] += 1
        self.every = every
        self._n = 0

    def invoke(self, value):
        self._n += 1
        if self._n % self.every == 0:
            with ThroughputSink._LOCK:
                ThroughputSink.STAMPS[self.key].append((self._n, time.perf_counter()))

    def rate(self, skip_fraction: float = 0.2) -> float | None:
        with ThroughputSink._LOCK:
            ts = sorted(ThroughputSink.STAMPS[self.key], key=lambda x: x[1])
        k = int(len(ts) * skip_fraction)
        if len(ts) < k + 2:
            return None
        return (ts[-1][0] - ts[k][0]) / (ts[-1][1] - ts[k][1])
