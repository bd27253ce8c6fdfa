"""DataStream API: ``StreamExecutionEnvironment``, ``DataStream``, ``KeyedStream``,
``ConnectedStreams``, windowed streams (the Flink 1.2 surface the reference programs use:
``readFile``, ``fromCollection``, ``map``/``flatMap``, ``keyBy``, windows, ``connect``,
``print``, ``execute``) plus ``map_with_model`` (``LIB/streaming/package.scala:15-43``)
and its micro-batched GPU variant ``map_with_model_batched``.
"""
from __future__ import annotations

import itertools
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable, Sequence

from . import functions as F
from .checkpoint import RestartStrategy
from .executor import LocalExecutor, Partitioner, clone_function
from .operators import (CoProcessOperator, CountWindows, FilterOperator, FlatMapOperator, MapOperator,
                        Operator, ProcessOperator, SinkOperator, SlidingEventTimeWindows, TimestampAssignerOperator,
                        TumblingEventTimeWindows, TumblingProcessingTimeWindows, UnionOperator, WindowAssigner,
                        WindowOperator)
from .sources import (CollectionSource, FileMonitoringSource, GeneratorSource, MemorySink, PrintSink,
                      PROCESS_ONCE, WholeFileInputFormat)

_uid = itertools.count()


@dataclass
class ExecutionConfig:
    channel_capacity: int = 1024
    registered_types: list = field(default_factory=list)
    global_job_parameters: dict = field(default_factory=dict)

    def register_type(self, t):
        if t not in self.registered_types:
            self.registered_types.append(t)

    @property
    def engine(self):
        """The job's :class:`~flink_tensorflow_amd.config.EngineConfig` (defaults if none)."""
        from ..config import EngineConfig

        e = self.global_job_parameters.get("engine")
        return e if e is not None else EngineConfig()


def register_types(config: ExecutionConfig) -> None:
    """``RegistrationUtils.registerTypes`` (``LIB/util/RegistrationUtils.java:18-86``):
    registers the TF protobuf message types and TensorValue with the job's type registry
    (they travel as length-prefixed protobuf bytes / TensorValue framing)."""
    from ..proto.messages import REGISTERED_TYPES
    from ..types.tensor_value import TensorValue

    for t in REGISTERED_TYPES + [TensorValue]:
        config.register_type(t)


class _Node:
    def __init__(self, name: str, factory: Callable[[], Operator], parallelism: int, inputs=None,
                 is_source: bool = False, uses_gpu: bool = False, wants_group: bool = False):
        self.uid = f"{next(_uid)}-{name}"
        self.name = name
        self.factory = factory
        self.parallelism = parallelism
        self.inputs: list[tuple[_Node, Partitioner, Any]] = inputs or []
        self.is_source = is_source
        self.uses_gpu = uses_gpu
        # the operator's subtasks run collectives (distributed weights, a DP trainer): with
        # the job communicator on "auto" only such operators form one (runtime/executor.py)
        self.wants_group = wants_group

    def make_operator(self) -> Operator:
        return self.factory()


class StreamExecutionEnvironment:
    _default_parallelism = 1

    def __init__(self):
        self.parallelism = StreamExecutionEnvironment._default_parallelism
        self.config = ExecutionConfig()
        self.nodes: list[_Node] = []
        self.checkpoint_interval: float | None = None
        self.checkpoint_dir: str | None = None
        self.restore_from_latest = False
        self.restart_strategy = RestartStrategy.no_restart()
        self.fault_injector = None
        self.chaining = True
        # one communicator per worker-process GPU operator (runtime/remote.py): "auto" forms it
        # when the operator runs P > 1 subtasks and the node has >= P GPUs; True also for P = 1
        # a splittable source (GeneratorSource: each subtask generates its own share) whose only
        # consumer is a worker-process operator of equal parallelism runs INSIDE the workers,
        # chained with it, instead of producing in the coordinator and shipping every record
        # across (executor.py ``_relocate_sources``)
        self.relocate_sources = True
        self.job_communicator: bool | str = "auto"
        self.test_communicator = None  # test-only injection (parallel/fake.py), never set by product code
        from ..parallel.comm import world

        self.rank, self.world_size, _ = world()

    @staticmethod
    def get_execution_environment() -> "StreamExecutionEnvironment":
        return StreamExecutionEnvironment()

    getExecutionEnvironment = get_execution_environment

    # ---- configuration
    def set_parallelism(self, p: int) -> "StreamExecutionEnvironment":
        self.parallelism = int(p)
        return self

    def get_parallelism(self) -> int:
        return self.parallelism

    def enable_job_communicator(self, on: bool | str = True, communicator=None) -> "StreamExecutionEnvironment":
        """Data parallelism inside one job: the P worker-process subtasks of a GPU operator
        form one communicator (RCCL over xGMI, subtask = rank, one GPU per subtask), so a
        model opened with ``distributed_weights=True`` is read by subtask 0 only and
        broadcast, and a ``ModelCoProcessFunction`` trainer all-reduces its gradients with
        ``parallel.comm.get()``.  ``communicator`` injects a test implementation."""
        self.job_communicator = on
        self.test_communicator = communicator
        return self

    def disable_operator_chaining(self) -> "StreamExecutionEnvironment":
        """Every operator runs in its own subtask thread (records cross a channel between
        any two operators); by default forward-connected operators are chained."""
        self.chaining = False
        return self

    disableOperatorChaining = disable_operator_chaining

    def get_config(self) -> ExecutionConfig:
        return self.config

    def enable_checkpointing(self, interval_s: float, directory: str, restore_from_latest: bool = False):
        self.checkpoint_interval = interval_s
        self.checkpoint_dir = directory
        self.restore_from_latest = restore_from_latest
        return self

    def set_restart_strategy(self, s: RestartStrategy):
        self.restart_strategy = s
        return self

    # ---- sources
    def add_source(self, fn: F.SourceFunction, name: str = "source", parallelism: int | None = None) -> "DataStream":
        proto = fn

        def factory():
            return Operator(clone_function(proto), name)

        node = _Node(name, factory, parallelism or self.parallelism, is_source=True)
        node.source_fn = proto  # inspected by the executor (worker-local source relocation)
        self.nodes.append(node)
        return DataStream(self, node)

    def from_collection(self, items: Iterable, timestamps: Sequence[float] | None = None,
                        parallelism: int = 1) -> "DataStream":
        return self.add_source(CollectionSource(list(items), timestamps), "collection", parallelism)

    fromCollection = from_collection

    def from_elements(self, *items) -> "DataStream":
        return self.from_collection(items)

    def generate(self, factory: Callable[[int, int, int], Iterable], limit: int | None = None,
                 parallelism: int | None = None, bulk: bool = False) -> "DataStream":
        """``factory(subtask, parallelism, start_record)`` yields the subtask's records — or,
        with ``bulk``, lists of records, each handed to the chained consumer as one run."""
        return self.add_source(GeneratorSource(factory, limit, bulk), "generator", parallelism)

    def read_file(self, fmt: WholeFileInputFormat, path: str, mode=PROCESS_ONCE, interval_s: float = 1.0,
                  parallelism: int | None = None, max_polls: int | None = None,
                  monitor: str = "coordinator", read_threads: int = 8) -> "DataStream":
        """``StreamExecutionEnvironment.readFile`` (``EX/inception/inception.scala:33-34``)
        as Flink builds it: one monitor (parallelism 1, in the coordinator) forwarding the
        new files' paths round-robin to ``parallelism`` readers (default: the
        environment's) that read and decode them.  A reader feeding a worker-process GPU
        operator of its parallelism is chained into that worker, so decoding happens where
        the records are consumed and only paths cross the coordinator.  ``monitor=
        "partitioned"``: each reader lists the directory itself and takes its hash share of the
        files (``sources.PartitionedFileSource``) — nothing crosses the coordinator."""
        from .operators import FileReaderOperator
        from .sources import FileMonitorFunction, PartitionedFileSource

        if monitor == "partitioned":
            # one listing + reading source subtask per reader (``PartitionedFileSource``):
            # relocated into the worker process of the operator it feeds, so nothing
            # crosses the coordinator
            return self.add_source(PartitionedFileSource(fmt, path, mode, interval_s, max_polls,
                                                         read_threads=read_threads), "file-source",
                                   parallelism or self.parallelism)
        if monitor != "coordinator":
            raise ValueError("read_file: monitor must be 'coordinator' or 'partitioned'")
        mon = self.add_source(FileMonitorFunction(fmt, path, mode, interval_s, max_polls), "file-monitor", 1)
        proto = fmt
        readers = mon._add("file-reader", lambda: FileReaderOperator(clone_function(proto), "file-reader"),
                           parallelism or self.parallelism, Partitioner("rebalance"))
        readers.node.chain_into_worker = True
        return readers

    readFile = read_file

    # ---- execution
    def _topo_nodes(self) -> list[_Node]:
        return list(self.nodes)

    def execute(self, job_name: str = "job"):
        return LocalExecutor(self, job_name).execute()


class DataStream:
    def __init__(self, env: StreamExecutionEnvironment, node: _Node):
        self.env = env
        self.node = node

    # ---- plumbing
    def _add(self, name: str, factory, parallelism=None, partitioner: Partitioner | None = None,
             uses_gpu: bool = False, extra_inputs=(), wants_group: bool = False) -> "DataStream":
        part = partitioner or Partitioner("forward")
        inputs = [(self.node, part, None)] + list(extra_inputs)
        node = _Node(name, factory, parallelism or self.env.parallelism, inputs, uses_gpu=uses_gpu,
                     wants_group=wants_group)
        self.env.nodes.append(node)
        return DataStream(self.env, node)

    def _edge_partitioner(self) -> Partitioner:
        return Partitioner("forward")

    def set_parallelism(self, p: int) -> "DataStream":
        self.node.parallelism = int(p)
        return self

    def run_in_processes(self, enable: bool = True) -> "DataStream":
        """Runs each subtask of this operator in its own worker process (one per GPU for
        model operators), fed through shared-memory rings (``runtime/remote.py``).

        On a source, the source subtasks run in the workers too, and every downstream
        operator that also runs in processes and is forward-connected with equal parallelism
        (single input, single consumer) is chained into the same worker: records are
        produced and consumed there and never cross the coordinator (a parallel source
        feeding one model worker per GPU)."""
        self.node.remote = bool(enable)
        return self

    def start_new_chain(self) -> "DataStream":
        """This operator starts a new chain: it is not chained into its upstream (its own
        downstream may still chain into it)."""
        self.node.chain_head = True
        return self

    def disable_chaining(self) -> "DataStream":
        """This operator is chained neither into its upstream nor with its downstream."""
        self.node.chaining = False
        return self

    startNewChain = start_new_chain
    disableChaining = disable_chaining

    def name(self, n: str) -> "DataStream":
        self.node.name = n
        return self

    def uid(self, u: str) -> "DataStream":
        self.node.uid = u
        return self

    # ---- partitioning
    def _repartition(self, kind: str, arg=None) -> "DataStream":
        ds = self._add(kind, lambda: UnionOperator(None, kind), partitioner=Partitioner(kind, arg))
        ds.node.passthrough = kind  # a pass-through node that only repartitions
        return ds

    def rebalance(self):
        return self._repartition("rebalance")

    def broadcast(self):
        return self._repartition("broadcast")

    def shuffle(self):
        return self._repartition("shuffle")

    def partition_custom(self, partitioner: Callable[[Any, int], int], key_selector: Callable) -> "DataStream":
        """``DataStream.partitionCustom(partitioner, keySelector)``: each record goes to
        channel ``partitioner(key_selector(record), num_channels)``."""
        return self._repartition("custom", (partitioner, key_selector))

    partitionCustom = partition_custom

    def global_(self):
        return self._repartition("global")

    def key_by(self, key_selector: Callable) -> "KeyedStream":
        return KeyedStream(self.env, self.node, key_selector)

    keyBy = key_by

    def union(self, *others: "DataStream") -> "DataStream":
        extra = [(o.node, Partitioner("forward"), None) for o in others]
        return self._add("union", lambda: UnionOperator(None, "union"), extra_inputs=extra)

    # ---- transformations
    def map(self, fn, name: str = "map", parallelism=None) -> "DataStream":
        proto = F.as_map(fn)
        return self._add(name, lambda: MapOperator(clone_function(proto), name), parallelism,
                         self._edge_partitioner(), uses_gpu=_uses_gpu(proto), wants_group=_wants_group(proto))

    def flat_map(self, fn, name: str = "flat-map", parallelism=None) -> "DataStream":
        proto = F.as_flat_map(fn)
        return self._add(name, lambda: FlatMapOperator(clone_function(proto), name), parallelism,
                         self._edge_partitioner(), uses_gpu=_uses_gpu(proto), wants_group=_wants_group(proto))

    flatMap = flat_map

    def filter(self, fn, name: str = "filter") -> "DataStream":
        proto = F.as_filter(fn)
        return self._add(name, lambda: FilterOperator(clone_function(proto), name), None, self._edge_partitioner())

    def process(self, fn: F.ProcessFunction, name: str = "process", parallelism=None) -> "DataStream":
        proto = fn
        return self._add(name, lambda: ProcessOperator(clone_function(proto), None, name), parallelism,
                         self._edge_partitioner(), uses_gpu=_uses_gpu(proto), wants_group=_wants_group(proto))

    def assign_timestamps_and_watermarks(self, extractor: Callable, max_out_of_orderness_s: float = 0.0):
        return self._add("timestamps", lambda: TimestampAssignerOperator(extractor, max_out_of_orderness_s))

    def connect(self, other: "DataStream") -> "ConnectedStreams":
        return ConnectedStreams(self, other)

    # ---- windows (non-keyed)
    def window_all(self, assigner: WindowAssigner) -> "AllWindowedStream":
        return AllWindowedStream(self, assigner)

    def count_window_all(self, n: int) -> "AllWindowedStream":
        return AllWindowedStream(self, CountWindows(n))

    def time_window_all(self, size_s: float, event_time: bool = False) -> "AllWindowedStream":
        return AllWindowedStream(self, TumblingEventTimeWindows(size_s) if event_time
                                 else TumblingProcessingTimeWindows(size_s))

    # ---- model integration (L6)
    def map_with_model(self, model, fun: Callable[[Any, Any], Any], name: str = "map-with-model",
                       parallelism=None) -> "DataStream":
        """``RichDataStream.mapWithModel`` (``LIB/streaming/package.scala:15-43``)."""
        if model is None:
            raise ValueError("model must not be None")
        if fun is None:
            raise ValueError("function must not be None")
        from .model_functions import ModelMapFunction

        return self.map(_LambdaModelMap(model, fun), name, parallelism)

    mapWithModel = map_with_model

    def flat_map_with_model(self, model, fun, name="flat-map-with-model", parallelism=None) -> "DataStream":
        if model is None or fun is None:
            raise ValueError("model and function must not be None")
        return self.flat_map(_LambdaModelFlatMap(model, fun), name, parallelism)

    def map_with_model_batched(self, model, batch_fn: Callable | None = None, max_batch: int = 64,
                               max_delay_ms: float = 5.0, name: str = "batched-model", parallelism=None,
                               emit_batches: bool = False) -> "DataStream":
        """Micro-batched model operator: records are staged into GPU micro-batches of up
        to ``max_batch`` (or whatever arrived within ``max_delay_ms``) and run through
        ``batch_fn(model, records) -> results`` — or, for models implementing
        ``BatchedGpuModel``, through the pipelined pinned-H2D / hipGraph runner.  Batches
        never straddle a checkpoint barrier (flushed before the snapshot)."""
        from .model_functions import BatchedModelOperator

        proto_model, proto_fn = model, batch_fn
        return self._add(name, lambda: BatchedModelOperator(clone_function(proto_model),
                                                            clone_function(proto_fn) if proto_fn else None,
                                                            max_batch, max_delay_ms, name, emit_batches),
                         parallelism, self._edge_partitioner(), uses_gpu=True,
                         wants_group=_wants_group(proto_model) or _wants_group(proto_fn))

    # ---- sinks
    def add_sink(self, fn, name: str = "sink", parallelism=None) -> "DataStream":
        proto = F.as_sink(fn)
        return self._add(name, lambda: SinkOperator(clone_function(proto), name), parallelism,
                         self._edge_partitioner())

    addSink = add_sink

    def print(self, prefix: str = "") -> "DataStream":
        return self.add_sink(PrintSink(prefix), "print")

    def collect_into(self, sink: MemorySink | None = None) -> MemorySink:
        sink = sink or MemorySink()
        self.add_sink(sink, "collect")
        return sink

    def execute_and_collect(self, job_name: str = "collect") -> list:
        sink = self.collect_into()
        self.env.execute(job_name)
        return sink.results()

    def get_side_output(self, tag: F.OutputTag) -> "DataStream":
        node = _Node(f"side-{tag.name}", lambda: UnionOperator(None, "side"), self.node.parallelism,
                     [(self.node, Partitioner("forward"), tag)])
        self.env.nodes.append(node)
        return DataStream(self.env, node)


class KeyedStream(DataStream):
    def __init__(self, env, node, key_selector):
        super().__init__(env, node)
        self.key_selector = key_selector

    def _edge_partitioner(self) -> Partitioner:
        return Partitioner("hash", self.key_selector)

    def process(self, fn: F.ProcessFunction, name: str = "keyed-process", parallelism=None) -> DataStream:
        proto, ks = fn, self.key_selector
        return self._add(name, lambda: ProcessOperator(clone_function(proto), ks, name), parallelism,
                         self._edge_partitioner(), uses_gpu=_uses_gpu(proto), wants_group=_wants_group(proto))

    def window(self, assigner: WindowAssigner) -> "WindowedStream":
        return WindowedStream(self, assigner)

    def count_window(self, n: int) -> "WindowedStream":
        return WindowedStream(self, CountWindows(n))

    def time_window(self, size_s: float, event_time: bool = False, slide_s: float | None = None):
        if slide_s is not None:
            return WindowedStream(self, SlidingEventTimeWindows(size_s, slide_s))
        return WindowedStream(self, TumblingEventTimeWindows(size_s) if event_time
                              else TumblingProcessingTimeWindows(size_s))

    def reduce(self, fn: Callable[[Any, Any], Any], name="reduce") -> DataStream:
        return self.process(_ReduceProcess(fn), name)


class ConnectedStreams:
    def __init__(self, a: DataStream, b: DataStream, k1=None, k2=None):
        self.a, self.b, self.k1, self.k2 = a, b, k1, k2

    def key_by(self, k1: Callable, k2: Callable) -> "ConnectedStreams":
        return ConnectedStreams(self.a, self.b, k1, k2)

    def process(self, fn: F.CoProcessFunction, name: str = "co-process", parallelism=None) -> DataStream:
        proto, k1, k2 = fn, self.k1, self.k2
        p1 = Partitioner("hash", k1) if k1 is not None else Partitioner("forward")
        p2 = Partitioner("hash", k2) if k2 is not None else Partitioner("forward")
        # the second input of an unkeyed co-process (e.g. a model-update stream) goes to every subtask
        if k2 is None:
            p2 = Partitioner("broadcast")
        return self.a._add(name, lambda: CoProcessOperator(clone_function(proto), k1, k2, name), parallelism, p1,
                           uses_gpu=_uses_gpu(proto), wants_group=_wants_group(proto),
                           extra_inputs=[(self.b.node, p2, None)])


class WindowedStream:
    def __init__(self, keyed: KeyedStream, assigner: WindowAssigner):
        self.keyed, self.assigner = keyed, assigner

    def apply(self, fn: F.WindowFunction, name: str = "window", parallelism=None) -> DataStream:
        proto, ks, asg = fn, self.keyed.key_selector, self.assigner
        return self.keyed._add(name, lambda: WindowOperator(clone_function(proto), asg, ks, False, name), parallelism,
                               self.keyed._edge_partitioner(), uses_gpu=_uses_gpu(proto),
                               wants_group=_wants_group(proto))

    def reduce(self, fn: Callable, name="window-reduce") -> DataStream:
        return self.apply(_ReduceWindow(fn), name)


class AllWindowedStream:
    def __init__(self, stream: DataStream, assigner: WindowAssigner):
        self.stream, self.assigner = stream, assigner

    def apply(self, fn: F.AllWindowFunction, name: str = "all-window") -> DataStream:
        proto, asg = fn, self.assigner
        return self.stream._add(name, lambda: WindowOperator(clone_function(proto), asg, None, True, name), 1,
                                Partitioner("global"), uses_gpu=_uses_gpu(proto), wants_group=_wants_group(proto))


# ------------------------------------------------------------------ helpers
def _uses_gpu(fn) -> bool:
    from .model_functions import ModelAwareFunction

    return isinstance(fn, ModelAwareFunction)


def _wants_group(obj) -> bool:
    """Does an operator's function (or its model) run collectives across its subtasks:
    ``distributed_weights`` (rank-0 read + broadcast at open) or ``uses_collectives`` (a
    data-parallel trainer: gradient all-reduce, sparse exchange)?"""
    for o in (obj, getattr(obj, "model", None), getattr(obj, "_model", None)):
        if o is not None and (getattr(o, "distributed_weights", False) or getattr(o, "uses_collectives", False)):
            return True
    return False


class _ReduceProcess(F.ProcessFunction):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def open(self, config=None):
        from .state import ValueStateDescriptor

        self.acc = self.get_runtime_context().get_state(ValueStateDescriptor("reduce"))

    def process_element(self, value, ctx, out):
        cur = self.acc.value()
        cur = value if cur is None else self.fn(cur, value)
        self.acc.update(cur)
        out.collect(cur)


class _ReduceWindow(F.WindowFunction):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def apply(self, key, window, inputs, out):
        it = iter(inputs)
        acc = next(it)
        for v in it:
            acc = self.fn(acc, v)
        out.collect(acc)


def _model_fn_classes():
    from .model_functions import ModelFlatMapFunction, ModelMapFunction

    return ModelMapFunction, ModelFlatMapFunction


class _LambdaModelMap:
    """Built lazily as a ModelMapFunction (import cycle avoidance)."""

    def __new__(cls, model, fun):
        ModelMapFunction, _ = _model_fn_classes()

        class _M(ModelMapFunction):
            def map(self, value):
                return fun(value, self.model)

        m = _M.__new__(_M)
        ModelMapFunction.__init__(m, model)
        return m


class _LambdaModelFlatMap:
    def __new__(cls, model, fun):
        _, ModelFlatMapFunction = _model_fn_classes()

        class _FM(ModelFlatMapFunction):
            def flat_map(self, value, out):
                r = fun(value, self.model)
                if r is not None:
                    for v in r:
                        out.collect(v)

        m = _FM.__new__(_FM)
        ModelFlatMapFunction.__init__(m, model)
        return m
