"""Stream operators: the per-subtask state machines wrapping user functions.

Element protocol (what travels on channels): ``Record(value, ts)``, ``Watermark(ts)``,
``Barrier(checkpoint_id)`` and ``EndOfInput``.  The task loop (``executor.py``) aligns
barriers across input channels and calls ``prepare_snapshot`` (flush micro-batches /
in-flight GPU work so a batch never straddles a barrier) → ``snapshot_state`` before
forwarding the barrier.
"""
from __future__ import annotations

import heapq
import time
from dataclasses import dataclass
from typing import Any, Callable

from .functions import (CheckpointedFunction, Collector, InitializationContext, OutputTag, ProcessContext,
                        RichFunction, RuntimeContext, SnapshotContext, TimeWindow)
from .state import KeyedStateStore, OperatorStateStore

# ------------------------------------------------------------------ stream elements


@dataclass
class Record:
    value: Any
    ts: float | None = None


@dataclass
class Watermark:
    ts: float


@dataclass
class Barrier:
    checkpoint_id: int
    timestamp: float = 0.0


class EndOfInput:
    __slots__ = ()


END = EndOfInput()


class Output:
    """Operator output: main stream + side outputs."""

    def __init__(self, emit: Callable[[Record], None], emit_side: Callable[[OutputTag, Any], None] | None = None,
                 emit_many: Callable[[list, Any], None] | None = None):
        self._emit = emit
        self._side = emit_side
        self._many = emit_many
        self.count = 0

    def emit(self, value, ts=None):
        self.count += 1
        self._emit(Record(value, ts))

    def emit_many(self, values: list, ts=None):
        """A run of values with one timestamp: handed over in one call where the consumer
        takes runs (a chained ``process_many``), else one ``emit`` each."""
        if self._many is not None:
            self.count += len(values)
            self._many(values, ts)
        else:
            for v in values:
                self.emit(v, ts)

    def emit_side(self, tag, value):
        if self._side is None:
            raise RuntimeError(f"no side output {tag.name!r} is consumed")
        self._side(tag, value)


# ------------------------------------------------------------------ base operator
class Operator:
    chainable = True
    num_inputs = 1

    def __init__(self, fn=None, name: str = "op"):
        self.fn = fn
        self.name = name
        self.ctx: RuntimeContext | None = None
        self.out: Output | None = None
        self.op_state = OperatorStateStore()
        self.keyed: KeyedStateStore | None = None
        self.current_timestamp = None
        self.current_key = None
        self.current_watermark = float("-inf")

    # lifecycle
    def setup(self, ctx: RuntimeContext, out: Output):
        self.ctx = ctx
        self.out = out

    def initialize(self, snapshot: dict | None, checkpoint_dir: str | None):
        if snapshot is not None:
            self.op_state = OperatorStateStore(snapshot.get("op"))
            if snapshot.get("keyed") is not None:
                self.keyed = KeyedStateStore(snapshot.get("keyed"))
            self.restore_extra(snapshot.get("extra"))
        if isinstance(self.fn, RichFunction):
            self.fn.set_runtime_context(self.ctx)
            if self.keyed is not None:
                self.ctx._keyed_state = self.keyed
        if isinstance(self.fn, CheckpointedFunction):
            self.fn.initialize_state(InitializationContext(self.op_state, snapshot is not None, checkpoint_dir,
                                                           self.ctx.subtask_index))

    def open(self):
        if isinstance(self.fn, RichFunction):
            self.fn.open(self.ctx.config)

    def close(self):
        if isinstance(self.fn, RichFunction):
            self.fn.close()

    # data
    def process(self, rec: Record, input_index: int = 0):
        raise NotImplementedError

    def process_batch(self, recs: list, input_index: int = 0):
        """The records of one channel message, in order (operators that gain from a run —
        the chained file reader — override this)."""
        for r in recs:
            self.process(r, input_index)

    def process_watermark(self, wm: Watermark, input_index: int = 0):
        self.current_watermark = max(self.current_watermark, wm.ts)
        self.on_watermark(self.current_watermark)
        self.out._emit(Watermark(self.current_watermark))

    def on_watermark(self, ts: float):  # noqa: B027
        pass

    def on_idle(self, now: float):  # noqa: B027
        """Called by the task loop when input is idle (processing-time triggers)."""

    def next_deadline(self) -> float | None:
        return None

    def end_input(self):  # noqa: B027
        """All inputs exhausted: flush pending work."""

    # checkpoints
    def prepare_snapshot(self):  # noqa: B027
        pass

    def snapshot_state(self, checkpoint_id: int, checkpoint_dir: str | None) -> dict:
        if isinstance(self.fn, CheckpointedFunction):
            self.fn.snapshot_state(SnapshotContext(checkpoint_id, time.time(), self.op_state, checkpoint_dir,
                                                   self.ctx.subtask_index))
        return {"op": self.op_state.snapshot(), "keyed": self.keyed.snapshot() if self.keyed else None,
                "extra": self.snapshot_extra()}

    def snapshot_extra(self):
        return None

    def restore_extra(self, extra):  # noqa: B027
        pass

    def notify_checkpoint_complete(self, checkpoint_id: int):
        f = getattr(self.fn, "notify_checkpoint_complete", None)
        if f is not None:
            f(checkpoint_id)


# ------------------------------------------------------------------ simple operators
class MapOperator(Operator):
    def process(self, rec, input_index=0):
        self.current_timestamp = rec.ts
        self.out.emit(self.fn.map(rec.value), rec.ts)


class FlatMapOperator(Operator):
    def setup(self, ctx, out):
        super().setup(ctx, out)
        self._ts = None
        self._col = Collector(lambda v: self.out.emit(v, self._ts))

    def process(self, rec, input_index=0):
        self._ts = rec.ts
        self.current_timestamp = rec.ts
        self.fn.flat_map(rec.value, self._col)


class FilterOperator(Operator):
    def process(self, rec, input_index=0):
        if self.fn.filter(rec.value):
            self.out.emit(rec.value, rec.ts)


class SinkOperator(Operator):
    def process(self, rec, input_index=0):
        self.current_timestamp = rec.ts
        self.fn.invoke(rec.value)


class TimestampAssignerOperator(Operator):
    """Assigns event timestamps and emits bounded-out-of-orderness watermarks."""

    def __init__(self, extractor, max_out_of_orderness: float = 0.0, name="timestamps"):
        super().__init__(None, name)
        self.extractor = extractor
        self.delay = max_out_of_orderness
        self.max_ts = float("-inf")

    def process(self, rec, input_index=0):
        ts = float(self.extractor(rec.value))
        self.max_ts = max(self.max_ts, ts)
        self.out.emit(rec.value, ts)
        wm = self.max_ts - self.delay
        if wm > self.current_watermark:
            self.current_watermark = wm
            self.out._emit(Watermark(wm))

    def process_watermark(self, wm, input_index=0):
        pass  # this operator generates watermarks

    def end_input(self):
        self.out._emit(Watermark(float("inf")))


# ------------------------------------------------------------------ timers
class TimerService:
    def __init__(self, op: "ProcessOperator"):
        self.op = op
        self.proc: list[tuple[float, Any]] = []
        self.event: list[tuple[float, Any]] = []

    def current_processing_time(self) -> float:
        return time.time()

    def current_watermark(self) -> float:
        return self.op.current_watermark

    def register_processing_time_timer(self, ts: float):
        heapq.heappush(self.proc, (ts, self.op.current_key))

    def register_event_time_timer(self, ts: float):
        heapq.heappush(self.event, (ts, self.op.current_key))

    def snapshot(self):
        return {"proc": list(self.proc), "event": list(self.event)}

    def restore(self, s):
        self.proc = list(s.get("proc", []))
        self.event = list(s.get("event", []))
        heapq.heapify(self.proc)
        heapq.heapify(self.event)


class ProcessOperator(Operator):
    """``ProcessFunction`` (optionally keyed) with processing/event-time timers."""

    def __init__(self, fn, key_selector=None, name="process"):
        super().__init__(fn, name)
        self.key_selector = key_selector
        if key_selector is not None:
            self.keyed = KeyedStateStore()
        self.timer_service = TimerService(self)

    def setup(self, ctx, out):
        super().setup(ctx, out)
        self._pctx = ProcessContext(self)
        self._col = Collector(lambda v: self.out.emit(v, self.current_timestamp))

    def _set_key(self, value):
        if self.key_selector is not None:
            self.current_key = self.key_selector(value)
            self.keyed.current_key = self.current_key

    def process(self, rec, input_index=0):
        self.current_timestamp = rec.ts
        self._set_key(rec.value)
        self.fn.process_element(rec.value, self._pctx, self._col)

    def emit_side(self, tag, value):
        self.out.emit_side(tag, value)

    def _fire(self, heap, limit):
        while heap and heap[0][0] <= limit:
            ts, key = heapq.heappop(heap)
            self.current_key = key
            if self.keyed is not None:
                self.keyed.current_key = key
            self.current_timestamp = ts
            self.fn.on_timer(ts, self._pctx, self._col)

    def on_watermark(self, ts):
        self._fire(self.timer_service.event, ts)

    def on_idle(self, now):
        self._fire(self.timer_service.proc, time.time())

    def next_deadline(self):
        return self.timer_service.proc[0][0] if self.timer_service.proc else None

    def _hook(self, name):
        f = getattr(self.fn, name, None)
        if f is not None:
            f(self._pctx, self._col)

    def open(self):
        super().open()
        self._hook("on_start")

    def prepare_snapshot(self):
        self._hook("on_barrier")

    def end_input(self):
        self._fire(self.timer_service.event, float("inf"))
        self._hook("on_end_of_input")

    def snapshot_extra(self):
        return {"timers": self.timer_service.snapshot()}

    def restore_extra(self, extra):
        if extra:
            self.timer_service.restore(extra.get("timers", {}))


class CoProcessOperator(ProcessOperator):
    num_inputs = 2
    chainable = False

    def __init__(self, fn, key1=None, key2=None, name="co-process"):
        super().__init__(fn, key1 or key2, name)
        self.keys = (key1, key2)

    def process(self, rec, input_index=0):
        self.current_timestamp = rec.ts
        ks = self.keys[input_index]
        if ks is not None:
            self.current_key = ks(rec.value)
            self.keyed.current_key = self.current_key
        if input_index == 0:
            self.fn.process_element1(rec.value, self._pctx, self._col)
        else:
            self.fn.process_element2(rec.value, self._pctx, self._col)


# ------------------------------------------------------------------ windows
class WindowAssigner:
    event_time = False

    def assign(self, value, ts, now) -> list:
        raise NotImplementedError


class TumblingProcessingTimeWindows(WindowAssigner):
    def __init__(self, size_s: float):
        self.size = size_s

    def assign(self, value, ts, now):
        start = now - (now % self.size)
        return [TimeWindow(start, start + self.size)]


class TumblingEventTimeWindows(WindowAssigner):
    event_time = True

    def __init__(self, size_s: float):
        self.size = size_s

    def assign(self, value, ts, now):
        if ts is None:
            raise ValueError("event-time windows need timestamps (assign_timestamps_and_watermarks)")
        start = ts - (ts % self.size)
        return [TimeWindow(start, start + self.size)]


class SlidingEventTimeWindows(WindowAssigner):
    event_time = True

    def __init__(self, size_s: float, slide_s: float):
        self.size, self.slide = size_s, slide_s

    def assign(self, value, ts, now):
        last = ts - (ts % self.slide)
        out = []
        s = last
        while s > ts - self.size:
            out.append(TimeWindow(s, s + self.size))
            s -= self.slide
        return out


class CountWindows(WindowAssigner):
    """Tumbling count window: fires every ``size`` elements per key."""

    def __init__(self, size: int):
        self.size = size

    def assign(self, value, ts, now):
        return ["count"]


class WindowOperator(Operator):
    def __init__(self, fn, assigner: WindowAssigner, key_selector=None, all_window=False, name="window",
                 allowed_lateness: float = 0.0):
        super().__init__(fn, name)
        self.assigner = assigner
        self.key_selector = key_selector
        self.all_window = all_window
        self.panes: dict[tuple, list] = {}
        self.lateness = allowed_lateness

    def setup(self, ctx, out):
        super().setup(ctx, out)
        self._col = Collector(lambda v: self.out.emit(v, self.current_timestamp))

    def process(self, rec, input_index=0):
        key = self.key_selector(rec.value) if self.key_selector is not None else None
        now = time.time()
        for w in self.assigner.assign(rec.value, rec.ts, now):
            if isinstance(w, TimeWindow) and self.assigner.event_time and w.end <= self.current_watermark - self.lateness:
                continue  # late element: dropped
            pane = self.panes.setdefault((key, w), [])
            pane.append(rec.value)
            if w == "count" and len(pane) >= self.assigner.size:
                self._fire(key, w)

    def _fire(self, key, w):
        items = self.panes.pop((key, w), [])
        if not items:
            return
        win = w if isinstance(w, TimeWindow) else None
        self.current_timestamp = win.end if win is not None else None
        if self.all_window:
            self.fn.apply(win, items, self._col)
        else:
            self.fn.apply(key, win, items, self._col)

    def _fire_until(self, limit):
        for (key, w) in sorted([k for k in self.panes if isinstance(k[1], TimeWindow) and k[1].end <= limit],
                               key=lambda k: k[1].end):
            self._fire(key, w)

    def on_watermark(self, ts):
        if self.assigner.event_time:
            self._fire_until(ts)

    def on_idle(self, now):
        if not self.assigner.event_time and not isinstance(self.assigner, CountWindows):
            self._fire_until(time.time())

    def next_deadline(self):
        if self.assigner.event_time or isinstance(self.assigner, CountWindows):
            return None
        ends = [w.end for (_, w) in self.panes if isinstance(w, TimeWindow)]
        return min(ends) if ends else None

    def end_input(self):
        for (key, w) in list(self.panes):
            self._fire(key, w)

    def snapshot_extra(self):
        return {"panes": {repr(k): (k, v) for k, v in self.panes.items()}}

    def restore_extra(self, extra):
        if extra:
            self.panes = {k: list(v) for k, v in extra.get("panes", {}).values()}


class UnionOperator(Operator):
    """Pass-through used to merge several inputs."""

    def process(self, rec, input_index=0):
        self.out._emit(rec)


# ------------------------------------------------------------------ file readers
class FileReaderOperator(Operator):
    """Flink's ``ContinuousFileReaderOperator``: receives file paths from the file monitor
    (``FileMonitorFunction``) and emits one record per file — ``fmt.read_record(path, bytes)`` (decode,
    normalise, the format's source-owned model) runs here, in the reader subtask, which the
    executor chains into the worker process of a GPU operator it feeds
    (``LocalExecutor._chain_into_workers``).  State: the splits received but not yet read
    (re-read after a restore), as Flink's reader keeps its pending splits."""

    def __init__(self, fmt, name: str = "file-reader"):
        super().__init__(None, name)
        self.fmt = fmt
        self.pending: list = []

    def open(self):
        self.fmt.open_input_format()
        self._drain(None)  # splits restored from a checkpoint

    def close(self):
        self.fmt.close_input_format()

    def process(self, rec: Record, input_index: int = 0):
        self.pending.append(rec.value)
        self._drain(rec.ts)

    def process_batch(self, recs: list, input_index: int = 0):
        """A message's run of paths: the local files are read on the native host pool in
        one call (GIL released) and the records go on as one run (``Output.emit_many``:
        one ``process_many`` of the chained model operator)."""
        from ..utils import fs

        self.pending.extend(r.value for r in recs)
        paths = list(self.pending)
        local = [fs.get_fs(p) for p in paths]
        if not all(isinstance(f, fs.LocalFS) for f, _ in local):
            return self._drain(recs[-1].ts if recs else None)
        from .. import _ext

        blobs = _ext.native().read_files([p for _, p in local], getattr(self, "read_threads", 8))
        outs = []
        for path, data in zip(paths, blobs):
            if data is None:  # unreadable: the per-file path raises with the OS error
                data = fs.read_bytes(path)
            out = self.fmt.read_record(path, data)
            if out is not None:
                outs.append(out)
        self.pending.clear()
        if outs:
            self.out.emit_many(outs, recs[-1].ts)

    def _drain(self, ts):
        from ..utils import fs

        while self.pending:
            path = self.pending[0]
            out = self.fmt.read_record(path, fs.read_bytes(path))
            self.pending.pop(0)
            if out is not None:
                self.out.emit(out, ts)

    def snapshot_extra(self):
        return {"pending": list(self.pending)}

    def restore_extra(self, extra):
        self.pending = list((extra or {}).get("pending", []))


class ChainOperator(Operator):
    """Operators run back to back in one subtask (Flink's operator chain) when the head
    must live where the tail runs: a file reader chained in front of the GPU operator in
    its worker process.  Elements and watermarks flow through direct calls; checkpoint
    hooks visit the members head first (so the head's flushed output reaches the next one
    before it snapshots); the state is the list of the members' states."""

    def __init__(self, ops: list, name: str = "chain"):
        super().__init__(None, name)
        self.ops = list(ops)

    @property
    def chainable(self):
        return all(getattr(o, "chainable", True) for o in self.ops)

    def setup(self, ctx, out: Output):
        super().setup(ctx, out)
        for a, b in zip(self.ops, self.ops[1:]):
            def fwd(elem, b=b):
                if isinstance(elem, Watermark):
                    b.process_watermark(elem, 0)
                else:
                    b.process(elem, 0)

            many = getattr(b, "process_many", None)  # e.g. the batched model operator
            a.setup(ctx, Output(fwd, out._side, many))
        self.ops[-1].setup(ctx, out)

    def initialize(self, snapshot, checkpoint_dir):
        states = (snapshot or {}).get("chain") if snapshot is not None else None
        for i, op in enumerate(self.ops):
            op.initialize(states[i] if states is not None else None, checkpoint_dir)

    def open(self):
        for op in self.ops:
            op.open()

    def close(self):
        for op in self.ops:
            op.close()

    def process(self, rec: Record, input_index: int = 0):
        self.ops[0].process(rec, input_index)

    def process_batch(self, recs: list, input_index: int = 0):
        self.ops[0].process_batch(recs, input_index)

    def process_watermark(self, wm: Watermark, input_index: int = 0):
        self.ops[0].process_watermark(wm, input_index)

    def on_idle(self, now: float):
        for op in self.ops:
            op.on_idle(now)

    def next_deadline(self):
        ds = [d for d in (op.next_deadline() for op in self.ops) if d is not None]
        return min(ds) if ds else None

    def end_input(self):
        for op in self.ops:
            op.end_input()

    def prepare_snapshot(self):
        for op in self.ops:
            op.prepare_snapshot()

    def snapshot_state(self, checkpoint_id: int, checkpoint_dir):
        return {"chain": [op.snapshot_state(checkpoint_id, checkpoint_dir) for op in self.ops]}

    def notify_checkpoint_complete(self, checkpoint_id: int):
        for op in self.ops:
            op.notify_checkpoint_complete(checkpoint_id)
