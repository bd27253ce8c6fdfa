"""User-function interfaces of the streaming runtime (the Flink DataStream function API the
reference builds on: ``RichMapFunction``, ``RichFlatMapFunction``, ``RichProcessFunction``,
``RichCoProcessFunction``, ``RichWindowFunction``, ``RichAllWindowFunction``,
``CheckpointedFunction``, ``SourceFunction``, ``SinkFunction``).
"""
from __future__ import annotations

import abc
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable


class RuntimeContext:
    """Per-subtask context handed to ``open``."""

    def __init__(self, task_name: str, subtask_index: int, parallelism: int, device=None, attempt: int = 0,
                 metrics=None, config=None, job=None):
        self.task_name = task_name
        self.subtask_index = subtask_index
        self.parallelism = parallelism
        self.device = device
        self.attempt = attempt
        self.restart_attempts: int | None = None  # the job's restart budget (None: not in a job)
        self.metrics = metrics
        self.config = config
        self._job = job
        self._keyed_state = None
        self._timer_service = None

    # Flink-style accessors
    def get_index_of_this_subtask(self) -> int:
        return self.subtask_index

    def get_number_of_parallel_subtasks(self) -> int:
        return self.parallelism

    def get_state(self, descriptor):
        if self._keyed_state is None:
            raise RuntimeError("keyed state is only available on keyed streams")
        return self._keyed_state.get_state(descriptor)

    def get_list_state(self, descriptor):
        return self.get_state(descriptor)

    def get_map_state(self, descriptor):
        return self.get_state(descriptor)

    def get_metric_group(self):
        return self.metrics


class Function:
    """Base of all user functions."""


class RichFunction(Function):
    def __init__(self):
        self._runtime_context: RuntimeContext | None = None

    def set_runtime_context(self, ctx: RuntimeContext):
        self._runtime_context = ctx

    def get_runtime_context(self) -> RuntimeContext:
        if getattr(self, "_runtime_context", None) is None:
            raise RuntimeError("runtime context not set (function not opened)")
        return self._runtime_context

    def open(self, config=None) -> None:  # noqa: B027
        pass

    def close(self) -> None:  # noqa: B027
        pass


class Collector:
    def __init__(self, emit: Callable[[Any], None]):
        self._emit = emit

    def collect(self, value) -> None:
        self._emit(value)

    def close(self):
        pass


class MapFunction(Function):
    @abc.abstractmethod
    def map(self, value):
        ...


class RichMapFunction(RichFunction, MapFunction):
    pass


class FlatMapFunction(Function):
    @abc.abstractmethod
    def flat_map(self, value, out: Collector) -> None:
        ...


class RichFlatMapFunction(RichFunction, FlatMapFunction):
    pass


class FilterFunction(Function):
    @abc.abstractmethod
    def filter(self, value) -> bool:
        ...


class ProcessContext:
    def __init__(self, op):
        self._op = op

    def timestamp(self):
        return self._op.current_timestamp

    def timer_service(self):
        return self._op.timer_service

    def get_current_key(self):
        return self._op.current_key

    def output(self, tag: "OutputTag", value):
        self._op.emit_side(tag, value)


class ProcessFunction(RichFunction):
    @abc.abstractmethod
    def process_element(self, value, ctx: ProcessContext, out: Collector) -> None:
        ...

    def on_timer(self, timestamp: float, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        pass

    # lifecycle hooks (extensions: an operator whose subtasks must act together — the
    # collective trainer of runtime/lockstep.py — needs to act at these points too)
    def on_start(self, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        """After ``open``, before the first element (timers may be registered here)."""

    def on_barrier(self, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        """A checkpoint barrier is aligned: called right before the snapshot."""

    def on_end_of_input(self, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        """Every input is exhausted (after the final event-time timers fired)."""


KeyedProcessFunction = ProcessFunction


class CoProcessFunction(RichFunction):
    @abc.abstractmethod
    def process_element1(self, value, ctx: ProcessContext, out: Collector) -> None:
        ...

    @abc.abstractmethod
    def process_element2(self, value, ctx: ProcessContext, out: Collector) -> None:
        ...

    def on_timer(self, timestamp: float, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        pass

    # lifecycle hooks (extensions: an operator whose subtasks must act together — the
    # collective trainer of runtime/lockstep.py — needs to act at these points too)
    def on_start(self, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        """After ``open``, before the first element (timers may be registered here)."""

    def on_barrier(self, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        """A checkpoint barrier is aligned: called right before the snapshot."""

    def on_end_of_input(self, ctx: ProcessContext, out: Collector) -> None:  # noqa: B027
        """Every input is exhausted (after the final event-time timers fired)."""


@dataclass(frozen=True)
class TimeWindow:
    start: float
    end: float

    def max_timestamp(self):
        return self.end


@dataclass(frozen=True)
class GlobalWindow:
    start: float = 0.0
    end: float = float("inf")


class WindowFunction(RichFunction):
    """``apply(key, window, inputs, out)`` (keyed windows)."""

    @abc.abstractmethod
    def apply(self, key, window, inputs: Iterable, out: Collector) -> None:
        ...


class AllWindowFunction(RichFunction):
    """``apply(window, inputs, out)`` (non-keyed windows)."""

    @abc.abstractmethod
    def apply(self, window, inputs: Iterable, out: Collector) -> None:
        ...


class SinkFunction(RichFunction):
    @abc.abstractmethod
    def invoke(self, value) -> None:
        ...


class SourceContext:
    """Handed to ``SourceFunction.run``; ``collect`` emits while holding the checkpoint lock."""

    def collect(self, value, timestamp: float | None = None) -> None:
        raise NotImplementedError

    def collect_many(self, values, timestamp: float | None = None) -> None:
        """Emits ``values`` in order (one lock hold; a chained micro-batching consumer takes
        them as one run — ``process_many`` — instead of one call chain per record)."""
        with self.checkpoint_lock:
            for v in values:
                self.collect(v, timestamp)

    def emit_watermark(self, ts: float) -> None:
        raise NotImplementedError

    @property
    def checkpoint_lock(self):
        raise NotImplementedError


class SourceFunction(RichFunction):
    @abc.abstractmethod
    def run(self, ctx: SourceContext) -> None:
        ...

    def cancel(self) -> None:  # noqa: B027
        pass


class CheckpointedFunction(abc.ABC):
    """``snapshotState`` / ``initializeState`` (Flink's ``CheckpointedFunction``)."""

    @abc.abstractmethod
    def snapshot_state(self, ctx: "SnapshotContext") -> None:
        ...

    @abc.abstractmethod
    def initialize_state(self, ctx: "InitializationContext") -> None:
        ...


@dataclass
class SnapshotContext:
    checkpoint_id: int
    timestamp: float
    operator_state: Any       # OperatorStateStore
    checkpoint_dir: str | None = None
    subtask_index: int = 0


@dataclass
class InitializationContext:
    operator_state: Any
    restored: bool
    checkpoint_dir: str | None = None
    subtask_index: int = 0
    extra: dict = field(default_factory=dict)

    def is_restored(self) -> bool:
        return self.restored


@dataclass(frozen=True)
class OutputTag:
    name: str


# ------------------------------------------------------------------ lambda adapters
class _LambdaMap(MapFunction):
    def __init__(self, fn):
        self.fn = fn

    def map(self, value):
        return self.fn(value)


class _LambdaFlatMap(FlatMapFunction):
    def __init__(self, fn):
        self.fn = fn

    def flat_map(self, value, out):
        r = self.fn(value)
        if r is not None:
            for v in r:
                out.collect(v)


class _LambdaFilter(FilterFunction):
    def __init__(self, fn):
        self.fn = fn

    def filter(self, value):
        return bool(self.fn(value))


class _LambdaSink(SinkFunction):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def invoke(self, value):
        self.fn(value)


def as_map(fn) -> MapFunction:
    return fn if isinstance(fn, MapFunction) else _LambdaMap(fn)


def as_flat_map(fn) -> FlatMapFunction:
    return fn if isinstance(fn, FlatMapFunction) else _LambdaFlatMap(fn)


def as_filter(fn) -> FilterFunction:
    return fn if isinstance(fn, FilterFunction) else _LambdaFilter(fn)


def as_sink(fn) -> SinkFunction:
    return fn if isinstance(fn, SinkFunction) else _LambdaSink(fn)
