"""Local job executor: subtasks as threads, bounded channels, partitioners, barrier
alignment, watermarks, end-of-input propagation, failure handling and restarts.

This stands in for the Flink 1.2 runtime the reference runs on (JobManager/TaskManager,
Netty data exchange, checkpoint barriers — SURVEY §1 L0).  One process executes the
whole job graph (like the reference's ``LocalFlinkMiniCluster``); in distributed mode
(one process per GPU under ``torch.distributed.run``) every rank executes the same graph
on its partition of the sources, and model operators bind ``cuda:LOCAL_RANK``.

GPU work releases the GIL (kernel launches, pinned copies, the C++ gather), so a
model-operator thread overlaps with source/sink threads.
"""
from __future__ import annotations

import logging
import queue
import threading
import time
import traceback
from collections import deque
from dataclasses import dataclass, field
from typing import Any

import cloudpickle

from ..utils.metrics import MetricGroup
from .checkpoint import CheckpointCoordinator, CheckpointStorage, RestartStrategy
from .functions import RuntimeContext, SourceContext
from .operators import END, Barrier, EndOfInput, Output, Record, Watermark

LOG = logging.getLogger("flink_tensorflow_amd.runtime")


class JobCancelled(Exception):
    pass


class JobExecutionException(RuntimeError):
    pass


# ------------------------------------------------------------------ partitioners
def stable_hash(key) -> int:
    import zlib

    if isinstance(key, int):
        return key & 0x7FFFFFFF
    if isinstance(key, bytes):
        return zlib.crc32(key)
    return zlib.crc32(repr(key).encode())


class Partitioner:
    kind = "forward"

    def __init__(self, kind: str = "forward", key_selector=None):
        self.kind = kind
        self.key_selector = key_selector
        self._rr = 0

    def select(self, rec: Record, n: int, my_index: int) -> list[int]:
        k = self.kind
        if k == "forward":
            return [my_index % n]
        if k == "rebalance":
            self._rr = (self._rr + 1) % n
            return [self._rr]
        if k == "hash":
            return [stable_hash(self.key_selector(rec.value)) % n]
        if k == "broadcast":
            return list(range(n))
        if k == "global":
            return [0]
        if k == "shuffle":
            import random

            return [random.randrange(n)]
        if k == "custom":  # key_selector = (partition(key, n) -> channel, key selector)
            fn, ks = self.key_selector
            c = int(fn(ks(rec.value), n))
            if not 0 <= c < n:
                raise ValueError(f"custom partitioner returned {c} for {n} channels")
            return [c]
        raise ValueError(k)

    def clone(self):
        return Partitioner(self.kind, self.key_selector)


# ------------------------------------------------------------------ channels
class InputGate:
    def __init__(self, capacity: int):
        self.q: queue.Queue = queue.Queue(maxsize=capacity)

    def put(self, ch: int, elem, cancel: threading.Event):
        while True:
            try:
                self.q.put((ch, elem), timeout=0.1)
                return
            except queue.Full:
                if cancel.is_set():
                    raise JobCancelled()


@dataclass
class _Edge:
    gate: InputGate
    channel: int          # channel id at the receiving gate
    subtask: int          # receiving subtask index


@dataclass
class _OutEdge:
    partitioner: Partitioner
    targets: list[_Edge]  # one per downstream subtask
    side_tag: Any = None


class RecordBuffer(list):
    """A network-buffer's worth of records for one channel (amortises queue hand-offs)."""

    __slots__ = ()


class RecordWriter:
    """Partitions records onto output channels.  Records are buffered per channel and
    shipped as ``RecordBuffer``s when ``buffer_size`` records accumulated, when
    ``buffer_timeout_s`` elapsed, or before any control element (order is preserved)."""

    def __init__(self, out_edges: list[_OutEdge], my_index: int, cancel: threading.Event, buffer_size: int = 64,
                 buffer_timeout_s: float = 0.01):
        self.out_edges = out_edges
        self.my_index = my_index
        self.cancel = cancel
        self.buffer_size = buffer_size
        self.timeout = buffer_timeout_s
        self._bufs: dict[tuple[int, int], RecordBuffer] = {}
        self._last_flush = time.perf_counter()
        # one lock for buffering AND channel puts: a background flush can never reorder a
        # buffer behind a barrier/watermark emitted by the owning task
        self._lock = threading.RLock()

    def emit(self, elem):
        control = not isinstance(elem, Record)
        with self._lock:
            if control:
                self._flush_locked()
            for ei, oe in enumerate(self.out_edges):
                if oe.side_tag is not None and not control:
                    continue  # side-output edges get records only via emit_side, but all control elements
                self._send(ei, oe, elem)
            if not control and time.perf_counter() - self._last_flush > self.timeout:
                self._flush_locked()

    def emit_side(self, tag, value):
        with self._lock:
            for ei, oe in enumerate(self.out_edges):
                if oe.side_tag == tag:
                    self._send(ei, oe, Record(value, None))

    def _send(self, ei, oe, elem):
        n = len(oe.targets)
        if isinstance(elem, Record):
            for i in oe.partitioner.select(elem, n, self.my_index):
                b = self._bufs.get((ei, i))
                if b is None:
                    b = self._bufs[(ei, i)] = RecordBuffer()
                b.append(elem)
                if len(b) >= self.buffer_size:
                    del self._bufs[(ei, i)]
                    t = oe.targets[i]
                    t.gate.put(t.channel, b, self.cancel)
        else:  # control elements go to every channel
            for t in oe.targets:
                t.gate.put(t.channel, elem, self.cancel)

    def _flush_locked(self):
        bufs, self._bufs = self._bufs, {}
        self._last_flush = time.perf_counter()
        for (ei, i), b in bufs.items():
            t = self.out_edges[ei].targets[i]
            t.gate.put(t.channel, b, self.cancel)

    def flush(self):
        with self._lock:
            self._flush_locked()


# ------------------------------------------------------------------ source context
class _SourceCtx(SourceContext):
    def __init__(self, task: "_SourceTask"):
        self.task = task
        self._lock = threading.RLock()

    @property
    def checkpoint_lock(self):
        return self._lock

    def collect(self, value, timestamp=None):
        task = self.task
        with self._lock:  # re-entrant: sources normally hold it already (chain timer excluded)
            task.check_trigger()
            task.head_emit(Record(value, timestamp))
        task.metrics.inc("records_out")

    def emit_watermark(self, ts):
        with self._lock:
            self.task.head_emit(Watermark(ts))


# ------------------------------------------------------------------ tasks
class _Task:
    def __init__(self, job: "LocalExecutor", node, subtask: int, writer: RecordWriter, restore: dict | None):
        self.job = job
        self.node = node
        self.subtask = subtask
        self.writer = writer
        self.restore = restore
        self.uid = node.uid
        self.metrics = MetricGroup(f"{node.name}[{subtask}]")
        self.thread: threading.Thread | None = None

    def runtime_context(self):
        dev = self.job.device_for(self.node, self.subtask)
        ctx = RuntimeContext(self.node.name, self.subtask, self.node.parallelism, dev, self.job.attempt, self.metrics,
                             self.job.config, self.job)
        ctx.global_index = self.job.rank * self.node.parallelism + self.subtask
        ctx.global_parallelism = self.job.world_size * self.node.parallelism
        env = getattr(self.job, "env", None)
        ctx.restart_attempts = env.restart_strategy.attempts if env is not None else 0
        return ctx

    def start(self):
        self.thread = threading.Thread(target=self._guarded, name=f"{self.node.name}-{self.subtask}", daemon=True)
        self.thread.start()

    def _guarded(self):
        done = False
        try:
            self.run()
            done = True
        except JobCancelled:
            pass
        except BaseException as e:  # noqa: BLE001
            self.job.fail(self, e, traceback.format_exc())
        finally:
            # only a task that ran to its end stops being expected by checkpoints: a failed
            # or cancelled task must not let an in-flight checkpoint complete without its
            # state (the restart would restore the sources' offsets but lose this task's)
            if done and self.job.coordinator is not None:
                for t in [self] + getattr(self, "chain", []):
                    self.job.coordinator.task_finished((t.uid, t.subtask), getattr(t, "final_state", None))

    def run(self):
        raise NotImplementedError


class _SourceTask(_Task):
    """A source subtask, with the operators chained into it (Flink chains a source with
    its forward, equal-parallelism consumers: records go from ``SourceContext.collect``
    straight into the first member's ``process`` on this thread, no queue hand-off).

    Chain members get their time-driven work (``on_idle``: a micro-batch whose
    ``max_delay`` expired, completed GPU batches) from the collect path at most every
    millisecond, and from a timer thread under the checkpoint lock while the source
    function is not emitting (Flink's processing-time service fires under the same lock)."""

    def __init__(self, job, node, subtask, writer, restore, chain: list | None = None):
        super().__init__(job, node, subtask, writer, restore)
        self.pending_trigger: deque[int] = deque()
        self.op = self.node.make_operator()
        self.chain = chain or []
        self.head_emit = writer.emit if writer is not None else None
        self._last_poll = time.perf_counter()

    def check_trigger(self):
        while self.pending_trigger:
            cid = self.pending_trigger.popleft()
            d = self.job.chk_dir(cid)
            self.job.ack(cid, (self.uid, self.subtask), self.op.snapshot_state(cid, d))
            for t in self.chain:  # in chain order: each flush reaches the next before it snapshots
                t.op.prepare_snapshot()
                self.job.ack(cid, (t.uid, t.subtask), t.op.snapshot_state(cid, d))
            self.writer.emit(Barrier(cid, time.time()))
        if self.job.cancel.is_set():
            raise JobCancelled()
        if self.chain:
            now = time.perf_counter()
            if now - self._last_poll >= 1e-3:
                self._poll_chain(now)

    def _poll_chain(self, now):
        self._last_poll = now
        wall = time.time()
        for t in self.chain:
            t.op.on_idle(wall)
        self.writer.flush()

    def _chain_timer(self, lock, stop: threading.Event):
        try:
            while True:
                with lock:
                    dls = [d for d in (t.op.next_deadline() for t in self.chain) if d is not None]
                wait = 0.01 if not dls else min(0.01, max(2e-4, min(dls) - time.time()))
                if stop.wait(wait):
                    return
                if time.perf_counter() - self._last_poll < wait:
                    continue  # the source is emitting: the collect path polls
                with lock:
                    if stop.is_set():
                        return
                    self._poll_chain(time.perf_counter())
        except BaseException as e:  # noqa: BLE001
            self.job.fail(self, e, traceback.format_exc())

    def run(self):
        fn = self.op.fn
        tasks = [self] + self.chain
        for i, t in enumerate(tasks):
            nxt = tasks[i + 1] if i + 1 < len(tasks) else None
            out = Output(_chain_emit(nxt), _drop_side) if nxt else Output(self.writer.emit, self.writer.emit_side)
            t.op.setup(t.runtime_context(), out)
            t.op.initialize(t.restore, self.job.restore_dir)
        for t in reversed(tasks):  # downstream first: ready before anything is emitted into it
            t.op.open()
        self.job.wait_all_opened()
        if self.chain:
            self.head_emit = _chain_emit(self.chain[0])
        sctx = _SourceCtx(self)
        stop = threading.Event()
        timer = None
        if self.chain:
            timer = threading.Thread(target=self._chain_timer, args=(sctx.checkpoint_lock, stop),
                                     name=f"{self.node.name}-{self.subtask}-timer", daemon=True)
            timer.start()
        try:
            fn.run(sctx)
            with sctx.checkpoint_lock:
                stop.set()
                self.check_trigger()
                # end-of-input offsets: later checkpoints restore this source as exhausted
                self.final_state = self.op.snapshot_state(-1, None)
            if timer is not None:
                timer.join()
                self.head_emit(Watermark(float("inf")))
                for t in self.chain:  # in chain order: each flush reaches the next operator
                    t.op.end_input()
        finally:
            stop.set()
            for t in tasks:
                t.op.close()
        self.writer.emit(Watermark(float("inf")))
        self.writer.emit(END)


class _RemoteSourceTask(_Task):
    """A source subtask running in a worker process together with its chained worker
    operators (``runtime/remote.py`` ``RemoteChainProxy``).  This coordinator thread only
    forwards checkpoint triggers and waits for the end of input; the proxy's drainer
    emits the chain's output, acks the members' snapshots and forwards barriers."""

    def __init__(self, job, node, subtask, writer, restore, chain: list):
        super().__init__(job, node, subtask, writer, restore)
        from .remote import RemoteChainProxy

        self.pending_trigger: deque[int] = deque()
        self.chain = chain
        self.op = RemoteChainProxy([node] + [t.node for t in chain], subtask, job)
        self.op.fn = self.op  # job.fail() cancels sources through ``op.fn.cancel()``
        for t in chain:  # members live in the worker: notifications go through the proxy
            t.op = _WorkerMember()

    def run(self):
        proxy = self.op
        proxy.setup(self.runtime_context(), Output(self.writer.emit, self.writer.emit_side))
        contexts = [self.runtime_context()] + [t.runtime_context() for t in self.chain]
        proxy.start_chain(contexts, [self.restore] + [t.restore for t in self.chain], self.job.restore_dir)
        self.job.wait_all_opened()
        try:
            def poll():
                while self.pending_trigger:
                    cid = self.pending_trigger.popleft()
                    proxy.trigger(cid, self.job.chk_dir(cid))
                if self.job.cancel.is_set():
                    proxy.cancel()
                    raise JobCancelled()

            self.final_state = proxy.wait_source_end(poll)
        except BaseException:
            proxy._shutdown()
            raise
        proxy.close()  # the drainer has re-emitted everything up to the source's end
        for t, m in zip(self.chain, getattr(proxy, "member_metrics", [])):
            t.op.worker_metrics = m
        self.writer.emit(END)


class _WorkerMember:
    """Stand-in operator of a chain member that runs inside a worker-process source chain."""

    worker_metrics = None

    def notify_checkpoint_complete(self, checkpoint_id):
        pass  # the chain's proxy notifies the whole worker chain once


class _ChainedTask(_Task):
    """A subtask chained into its upstream subtask's thread (Flink's operator chaining:
    forward edge, equal parallelism, single input, single consumer).  It has no thread and
    no input gate: the chain's head task calls its operator directly, records never cross
    a queue, and it still has its own metrics, state snapshots and checkpoint acks."""

    def __init__(self, job, node, subtask, restore, op):
        super().__init__(job, node, subtask, None, restore)
        self.op = op

    def start(self):
        pass


def _chain_emit(task: _Task):
    op, inc = task.op, task.metrics.inc

    def emit(elem):
        if type(elem) is Record:
            inc("records_in")
            op.process(elem, 0)
        elif isinstance(elem, Watermark):
            op.process_watermark(elem, 0)
        else:
            raise TypeError(f"operators emit records and watermarks, not {type(elem).__name__}")

    return emit


def _drop_side(tag, value):
    pass  # no consumer of this side output (as for an unchained operator's writer)


class _OpTask(_Task):
    def __init__(self, job, node, subtask, writer, restore, gate: InputGate, channels: list[int], op=None,
                 chain: list[_ChainedTask] | None = None):
        super().__init__(job, node, subtask, writer, restore)
        self.gate = gate
        self.channel_input = dict(channels)  # channel id -> input index
        self.chain = chain or []
        if getattr(self.node, "remote", False):
            from .remote import RemoteOperatorProxy

            self.op = RemoteOperatorProxy(self.node, subtask, job)  # subtask runs in a worker process
        else:
            self.op = op if op is not None else self.node.make_operator()

    def run(self):
        op = self.op
        tasks = [self] + self.chain
        for i, t in enumerate(tasks):
            nxt = tasks[i + 1] if i + 1 < len(tasks) else None
            out = Output(_chain_emit(nxt), _drop_side) if nxt else Output(self.writer.emit, self.writer.emit_side)
            t.op.setup(t.runtime_context(), out)
            t.op.initialize(t.restore, self.job.restore_dir)
        for t in reversed(tasks):  # downstream first: ready before anything is emitted into it
            t.op.open()
        self.job.wait_all_opened()
        ops = [t.op for t in tasks]
        channels = set(self.channel_input)
        finished: set[int] = set()
        wms = {c: float("-inf") for c in channels}
        cur_wm = float("-inf")
        aligning: int | None = None
        arrived: set[int] = set()
        blocked_buf: dict[int, deque] = {c: deque() for c in channels}
        replay: deque = deque()
        cancel = self.job.cancel
        try:
            while True:
                if cancel.is_set():
                    raise JobCancelled()
                if not replay and finished >= channels:
                    # checked at the top of every iteration: the last EndOfInput may have
                    # completed an alignment whose blocked records were replayed since
                    for o in ops:  # in chain order: each flush reaches the next operator
                        o.end_input()
                    break
                if replay:
                    ch, elem = replay.popleft()
                else:
                    dls = [d for d in (o.next_deadline() for o in ops) if d is not None]
                    timeout = 0.05 if not dls else max(0.0, min(0.05, min(dls) - time.time()))
                    try:
                        ch, elem = self.gate.q.get(timeout=timeout)
                    except queue.Empty:
                        self.writer.flush()
                        now = time.time()
                        for o in ops:
                            o.on_idle(now)
                        continue
                if aligning is not None and ch in arrived:
                    # a channel past its barrier is blocked until the alignment completes,
                    # its EndOfInput included (so it is processed after its records)
                    blocked_buf[ch].append((ch, elem))
                    continue
                if isinstance(elem, RecordBuffer):
                    idx = self.channel_input[ch]
                    for r in elem:
                        op.process(r, idx)
                    self.metrics.inc("records_in", len(elem))
                elif isinstance(elem, Record):
                    op.process(elem, self.channel_input[ch])
                    self.metrics.inc("records_in")
                elif isinstance(elem, Watermark):
                    wms[ch] = max(wms[ch], elem.ts)
                    live = [wms[c] for c in channels if c not in finished] or [float("inf")]
                    m = min(live)
                    if m > cur_wm:
                        cur_wm = m
                        op.process_watermark(Watermark(m))
                elif isinstance(elem, Barrier):
                    if aligning is None:
                        aligning = elem.checkpoint_id
                        arrived = set()
                    arrived.add(ch)
                    if arrived | finished >= channels:
                        self._complete_barrier(elem)
                        aligning = None
                        for c in channels:
                            replay.extend(blocked_buf[c])
                            blocked_buf[c].clear()
                        arrived = set()
                elif isinstance(elem, EndOfInput):
                    finished.add(ch)
                    if aligning is not None and arrived | finished >= channels:
                        self._complete_barrier(Barrier(aligning))
                        aligning = None
                        for c in channels:
                            replay.extend(blocked_buf[c])
                            blocked_buf[c].clear()
                        arrived = set()
                now = time.time()
                for o in ops:
                    o.on_idle(now)
        finally:
            for o in ops:
                o.close()
        self.writer.emit(Watermark(float("inf")))
        self.writer.emit(END)

    def _complete_barrier(self, b: Barrier):
        # in chain order: an operator's pre-snapshot flush reaches the next one before
        # that one snapshots, so the chain's state is consistent at the barrier
        for t in [self] + self.chain:
            t.op.prepare_snapshot()
            state = t.op.snapshot_state(b.checkpoint_id, self.job.chk_dir(b.checkpoint_id))
            self.job.ack(b.checkpoint_id, (t.uid, t.subtask), state)
        self.writer.emit(b)


# ------------------------------------------------------------------ executor
@dataclass
class JobExecutionResult:
    job_name: str
    runtime_s: float
    attempts: int
    checkpoints: list[int] = field(default_factory=list)
    metrics: dict = field(default_factory=dict)

    def get_net_runtime(self):
        return self.runtime_s


class LocalExecutor:
    def __init__(self, env, job_name: str):
        self.env = env
        self.job_name = job_name
        self.config = env.config
        self.cancel = threading.Event()
        self.error: tuple | None = None
        self.tasks: list[_Task] = []
        self.sources: list[_SourceTask] = []
        self.coordinator: CheckpointCoordinator | None = None
        self.attempt = 0
        self.restore_dir: str | None = None
        self.rank, self.world_size = env.rank, env.world_size
        self._lock = threading.Lock()
        self._opened: threading.Barrier | None = None
        self._groups: dict = {}

    def operator_group(self, node) -> dict | None:
        """The rendezvous of a worker-process GPU operator's subtasks (one
        subtask per GPU, rank 0 loads, RCCL broadcast): a key/value store hosted here in the
        coordinator, under an attempt-scoped prefix.  Each worker opens its communicator on
        it (subtask = rank) before ``op.open()``; rank 0 publishes the RCCL unique id.  None
        when the operator does not form one: SPMD jobs (each rank runs its own subtasks
        and already has the global communicator), host operators, operators that run no
        collectives under the default "auto" mode (pure inference without
        ``distributed_weights``), or fewer GPUs than subtasks (RCCL needs one GPU per rank).  GPUs are counted from sysfs: the
        coordinator never initialises HIP for this."""
        mode = getattr(self.env, "job_communicator", "auto")
        test_cls = getattr(self.env, "test_communicator", None)
        if not mode or self.world_size > 1 or not node.uses_gpu:
            return None
        if mode == "auto" and (node.parallelism <= 1 or not getattr(node, "wants_group", False)):
            return None  # "auto": only operators that run collectives pay for an RCCL group
        if test_cls is None:
            from ..utils.gpus import sysfs_gpu_count

            if sysfs_gpu_count() < node.parallelism:
                return None
        with self._lock:
            g = self._groups.get(node.uid)
            if g is None:
                import datetime

                from torch.distributed import TCPStore

                store = TCPStore("127.0.0.1", 0, is_master=True, wait_for_workers=False,
                                 timeout=datetime.timedelta(seconds=600))
                g = self._groups[node.uid] = {"addr": "127.0.0.1", "port": store.port, "size": node.parallelism,
                                              "prefix": f"ftm-op/{node.uid}/{self.attempt}/",
                                              "cls": cloudpickle.dumps(test_cls) if test_cls is not None else None,
                                              "_store": store}
        return {k: v for k, v in g.items() if not k.startswith("_")}

    def wait_all_opened(self):
        """Start barrier: a task thread emits or processes its first record only after
        every task thread of the attempt has opened its operators.  GPU subtasks that share
        this process compile and capture their hipGraphs in ``open()``; without the barrier
        one subtask replays (and allocates, frees pinned blocks, runs the GC) on its streams
        while a sibling is still inside a stream capture, which the HIP runtime does not
        isolate per thread (``test_remote_batched_resnet_gpu``, round-3 driver abort)."""
        b = self._opened
        if b is None:
            return
        try:
            b.wait()
        except threading.BrokenBarrierError:
            raise JobCancelled() from None

    # ---- device binding: one model subtask per GPU
    def device_for(self, node, subtask):
        import torch

        if not node.uses_gpu or not torch.cuda.is_available():
            return None
        from ..parallel.comm import gpu_count

        n = max(1, gpu_count())
        if self.world_size > 1:
            import os

            return torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
        return torch.device("cuda", subtask % n)

    def chk_dir(self, cid):
        if self.coordinator is None:
            return None
        return self.coordinator.storage.chk_dir(cid)

    # ---- checkpoint plumbing
    def trigger_sources(self, cid):
        for s in self.sources:
            s.pending_trigger.append(cid)

    def ack(self, cid, task, state):
        if self.coordinator is not None:
            self.coordinator.acknowledge(cid, task, state)

    def notify_complete(self, cid):
        for t in self.tasks:
            try:
                t.op.notify_checkpoint_complete(cid)
            except Exception:  # noqa: BLE001
                LOG.exception("notify_checkpoint_complete failed")

    def fail(self, task, exc, tb):
        with self._lock:
            if self.error is None:
                self.error = (task, exc, tb)
        LOG.error("task %s[%d] failed: %s", task.node.name, task.subtask, exc)
        if self.coordinator is not None:
            self.coordinator.abort_pending()  # no checkpoint of a failed attempt may complete
        self.cancel.set()
        if self._opened is not None:
            self._opened.abort()  # tasks still waiting for their siblings' open() give up
        for s in self.sources:
            try:
                s.op.fn.cancel()
            except Exception:  # noqa: BLE001
                pass

    # ---- build + run
    def _build(self, restore_states: dict | None):
        self._groups = {}  # a restarted attempt rendezvouses afresh (new store, new prefix)
        nodes = self._chain_into_workers(self.env._topo_nodes())
        self.relocated = self._relocate_sources(nodes)
        cap = self.config.channel_capacity
        ops = {(n.uid, i): n.make_operator() for n in nodes if not n.is_source and not getattr(n, "remote", False)
               for i in range(n.parallelism)}
        chained_to = self._chains(nodes, ops)  # downstream uid -> upstream node it runs inside
        remote_chained = self._remote_source_chains(nodes)  # chained into a worker-process source
        chained_to.update(remote_chained)
        gates: dict[tuple[str, int], InputGate] = {}
        chan_of: dict[tuple[str, int], list] = {}
        for n in nodes:
            if not n.is_source and n.uid not in chained_to:
                for i in range(n.parallelism):
                    gates[(n.uid, i)] = InputGate(cap)
                    chan_of[(n.uid, i)] = []
        out_edges: dict[tuple[str, int], list[_OutEdge]] = {(n.uid, i): [] for n in nodes for i in range(n.parallelism)}
        for n in nodes:
            if n.uid in chained_to:
                continue  # fed by direct calls from its upstream operator
            for input_index, (up, part, side_tag) in enumerate(n.inputs):
                for ui in range(up.parallelism):
                    targets = []
                    for di in range(n.parallelism):
                        ch = len(chan_of[(n.uid, di)])
                        chan_of[(n.uid, di)].append((ch, input_index))
                        targets.append(_Edge(gates[(n.uid, di)], ch, di))
                    p = part.clone()
                    if p.kind == "forward" and up.parallelism != n.parallelism:
                        p = Partitioner("rebalance")
                    out_edges[(up.uid, ui)].append(_OutEdge(p, targets, side_tag))
        self.tasks, self.sources = [], []
        self.chains = []
        succ = {up.uid: n for n, up in ((n, chained_to[n.uid]) for n in nodes if n.uid in chained_to)}
        for n in nodes:
            if n.uid in chained_to:
                continue  # built with its chain's head
            members = []
            m = succ.get(n.uid)
            while m is not None:
                members.append(m)
                m = succ.get(m.uid)
            if members:
                self.chains.append([n.name] + [m.name for m in members])
            tail = members[-1] if members else n
            for i in range(n.parallelism):
                w = RecordWriter(out_edges[(tail.uid, i)], i, self.cancel)
                rs = restore_states.get((n.uid, i)) if restore_states else None
                if n.is_source and getattr(n, "remote", False):
                    chain = [_ChainedTask(self, m, i, restore_states.get((m.uid, i)) if restore_states else None, None)
                             for m in members]
                    t = _RemoteSourceTask(self, n, i, w, rs, chain)
                    self.sources.append(t)
                    self.tasks.append(t)
                    self.tasks.extend(chain)
                    continue
                chain = [_ChainedTask(self, m, i, restore_states.get((m.uid, i)) if restore_states else None,
                                      ops[(m.uid, i)] if (m.uid, i) in ops else self._remote_proxy(m, i))
                         for m in members]
                if n.is_source:
                    t = _SourceTask(self, n, i, w, rs, chain)
                    self.sources.append(t)
                    self.tasks.append(t)
                    self.tasks.extend(chain)
                    continue
                self.tasks.append(_OpTask(self, n, i, w, rs, gates[(n.uid, i)], chan_of[(n.uid, i)],
                                          ops.get((n.uid, i)), chain))
                self.tasks.extend(chain)

    def _remote_proxy(self, node, subtask):
        from .remote import RemoteOperatorProxy

        return RemoteOperatorProxy(node, subtask, self)

    def _chain_into_workers(self, nodes) -> list:
        """Chains a host operator marked ``chain_into_worker`` (``read_file``'s readers) into
        the worker process of the worker-process operator it feeds — same parallelism,
        forward or rebalance edge, that operator's only input: the worker then runs
        ``ChainOperator([reader, op])``, so files are read and decoded where their records
        are consumed and the coordinator sends only the monitor's paths (Flink chains the
        ``ContinuousFileReaderOperator`` with its successor in one task slot).  Idempotent
        across restart attempts.  Returns the nodes left to schedule."""
        from .operators import ChainOperator

        if not getattr(self.env, "chaining", True):
            return list(nodes)
        consumers: dict[str, list] = {}
        for n in nodes:
            for up, part, side_tag in n.inputs:
                consumers.setdefault(up.uid, []).append((n, part, side_tag))
        for r in nodes:
            if not getattr(r, "chain_into_worker", False) or getattr(r, "merged_into", None) is not None:
                continue
            cs = consumers.get(r.uid, [])
            if len(cs) != 1:
                continue
            d, part, side_tag = cs[0]
            skipped = []
            # a rebalance / shuffle right after the readers (``read_file(...).rebalance()``) only
            # spreads records the readers already spread: chained, the records are produced
            # in the consumer's worker and the repartition has nothing to move
            while (getattr(d, "passthrough", None) in ("rebalance", "shuffle") and side_tag is None
                   and len(consumers.get(d.uid, [])) == 1):
                skipped.append(d)
                d, part, side_tag = consumers[d.uid][0]
                part = Partitioner("rebalance") if part.kind == "forward" else part
            if (not getattr(d, "remote", False) or d.is_source or side_tag is not None or len(d.inputs) != 1
                    or d.parallelism != r.parallelism or part.kind not in ("forward", "rebalance")
                    or not getattr(d, "chaining", True)):
                continue
            head, tail, name = r.factory, d.factory, d.name
            d.factory = lambda head=head, tail=tail, name=name: ChainOperator([head(), tail()], name)
            d.inputs = list(r.inputs)
            r.merged_into = d
            for n in skipped:
                n.merged_into = d
        return [n for n in nodes if getattr(n, "merged_into", None) is None]

    def _relocate_sources(self, nodes) -> list[str]:
        """Moves relocatable sources into the worker processes of their consumer: a source
        whose function is splittable by subtask (``relocatable``), feeding exactly one
        worker-process operator of the same parallelism (forward or rebalance edge, single
        input), becomes a worker-process source chained with that operator — each worker
        produces its own share of the records where they are consumed, instead of the
        coordinator producing every record and copying it across (a rebalance between
        equal-parallelism splits becomes forward: each split's records stay with their
        worker, which is the even distribution rebalance asks for).  Returns the relocated
        source names."""
        if not getattr(self.env, "relocate_sources", True) or self.world_size > 1:
            return []
        consumers: dict[str, list] = {}
        for n in nodes:
            for i, (up, part, side_tag) in enumerate(n.inputs):
                consumers.setdefault(up.uid, []).append((n, i, part, side_tag))
        moved = []
        for src in nodes:
            fn = getattr(src, "source_fn", None)
            if not src.is_source or getattr(src, "remote", False) or not getattr(fn, "relocatable", False):
                continue
            path = [src]  # src -> [rebalance pass-through] -> worker operator
            ok = True
            while ok:
                cs = consumers.get(path[-1].uid, [])
                if len(cs) != 1:
                    ok = False
                    break
                dst, i, part, side_tag = cs[0]
                ok = (side_tag is None and len(dst.inputs) == 1 and dst.parallelism == src.parallelism
                      and part.kind in ("forward", "rebalance") and getattr(dst, "chaining", True)
                      and not getattr(dst, "chain_head", False))
                if not ok:
                    break
                path.append(dst)
                if getattr(dst, "remote", False):
                    break
                if getattr(dst, "passthrough", None) != "rebalance":
                    ok = False
            if not ok or not getattr(path[-1], "remote", False):
                continue
            for a, b in zip(path, path[1:]):  # forward edges, every hop in the worker
                up, part, side_tag = b.inputs[0]
                if part.kind != "forward":
                    b.inputs[0] = (up, Partitioner("forward"), side_tag)
                a.remote = True
            src.relocated = True
            moved.append(src.name)
        return moved

    def _remote_source_chains(self, nodes) -> dict:
        """Worker-process sources: the downstream worker operators they run together with
        (forward edge, equal parallelism, single input, single consumer, chaining allowed)
        — ``member uid -> upstream node``."""
        consumers: dict[str, int] = {}
        for n in nodes:
            for up, _, _ in n.inputs:
                consumers[up.uid] = consumers.get(up.uid, 0) + 1
        out = {}
        for src in nodes:
            if not (src.is_source and getattr(src, "remote", False)):
                continue
            cur = src
            while consumers.get(cur.uid) == 1:
                nxt = next(n for n in nodes if any(up is cur for up, _, _ in n.inputs))
                if len(nxt.inputs) != 1:
                    break
                up, part, side_tag = nxt.inputs[0]
                if not (getattr(nxt, "remote", False) and side_tag is None and part.kind == "forward"
                        and nxt.parallelism == cur.parallelism and getattr(nxt, "chaining", True)
                        and not getattr(nxt, "chain_head", False)):
                    break
                out[nxt.uid] = cur
                cur = nxt
        return out

    def _chains(self, nodes, ops) -> dict:
        """Operator chaining (Flink's ``StreamingJobGraphGenerator.isChainable``): a node runs
        inside its upstream's thread when the edge is forward, both have the same
        parallelism, it has exactly that one input, the upstream has no other consumer, and
        neither side is an operator that cannot chain (two-input) or a node marked
        ``start_new_chain`` / ``disable_chaining``.  A source heads a chain (``_SourceTask``
        runs its members), it never joins one; a worker-process operator's proxy is never
        chained (its own thread overlaps the slab scatter with the upstream's work)."""
        if not getattr(self.env, "chaining", True):
            return {}
        consumers: dict[str, int] = {}
        for n in nodes:
            for up, _, _ in n.inputs:
                consumers[up.uid] = consumers.get(up.uid, 0) + 1

        def ok(n, head=False):
            if not getattr(n, "chaining", True):
                return False
            if getattr(n, "remote", False):
                # a worker-process operator's proxy keeps its own thread: chained behind its
                # upstream, the record production and the slab scatter serialise on one thread
                # (measured: 2-3x less transport, profiles/r03_transport); remote sources chain
                # inside their worker instead (_remote_source_chains)
                return False
            if n.is_source:  # a source heads a chain; it never joins one
                return head
            return ops[(n.uid, 0)].chainable

        out = {}
        for n in nodes:
            if len(n.inputs) != 1 or getattr(n, "chain_head", False):
                continue
            up, part, side_tag = n.inputs[0]
            if (side_tag is None and part.kind == "forward" and up.parallelism == n.parallelism
                    and consumers.get(up.uid) == 1 and ok(up, head=True) and ok(n)):
                out[n.uid] = up
        return out

    def execute(self) -> JobExecutionResult:
        t0 = time.time()
        strategy: RestartStrategy = self.env.restart_strategy
        storage = CheckpointStorage(self.env.checkpoint_dir) if self.env.checkpoint_dir else None
        restore_states = None
        if storage is not None and self.env.restore_from_latest and storage.latest() is not None:
            restore_states = storage.load(storage.latest())
            self.restore_dir = storage.chk_dir(storage.latest())
        completed = []
        while True:
            self.cancel.clear()
            self.error = None
            self._build(restore_states)
            if storage is not None and self.env.checkpoint_interval:
                self.coordinator = CheckpointCoordinator(storage, self.env.checkpoint_interval, self)
                self.coordinator.start({(t.uid, t.subtask) for t in self.tasks})
            if self.env.fault_injector is not None:
                self.env.fault_injector.arm(self)
            self._opened = threading.Barrier(sum(1 for t in self.tasks if not isinstance(t, _ChainedTask)))
            for t in self.tasks:
                t.start()
            stop_flush = threading.Event()

            def flusher(srcs=list(self.sources)):
                # sources may block between records (file monitor intervals, rate limits):
                # ship their partially filled buffers on the buffer timeout
                while not stop_flush.wait(0.005):
                    for s in srcs:
                        try:
                            s.writer.flush()
                        except JobCancelled:
                            return

            fl = threading.Thread(target=flusher, name="buffer-flusher", daemon=True)
            fl.start()
            for t in self.tasks:
                while t.thread is not None and t.thread.is_alive():
                    t.thread.join(timeout=0.2)
                    if self.error is not None:
                        break
            if self.error is not None:
                for t in self.tasks:
                    if t.thread is not None:
                        t.thread.join(timeout=5)
            stop_flush.set()
            fl.join(timeout=1)
            if self.coordinator is not None:
                self.coordinator.stop()
                completed += self.coordinator.completed_ids
            if self.error is None:
                break
            task, exc, tb = self.error
            if self.attempt >= strategy.attempts:
                raise JobExecutionException(f"job {self.job_name!r} failed in {task.node.name}[{task.subtask}]: "
                                            f"{exc}\n{tb}") from exc
            self.attempt += 1
            LOG.warning("restarting job %s (attempt %d/%d) after: %s", self.job_name, self.attempt,
                        strategy.attempts, exc)
            time.sleep(strategy.delay_s)
            restore_states = None
            self.restore_dir = None
            if storage is not None and storage.latest() is not None:
                restore_states = storage.load(storage.latest())
                self.restore_dir = storage.chk_dir(storage.latest())
        metrics = {f"{t.node.name}[{t.subtask}]": _task_metrics(t) for t in self.tasks}
        return JobExecutionResult(self.job_name, time.time() - t0, self.attempt, completed, metrics)


def _task_metrics(task) -> dict:
    """The task's metrics; a worker-process subtask adds what its operator recorded in the
    worker (latency / batch-size histograms, operator counters)."""
    snap = task.metrics.snapshot()
    w = getattr(getattr(task, "op", None), "worker_metrics", None)
    if w:
        for section in ("histograms", "gauges", "rates"):
            snap.setdefault(section, {}).update(w.get(section, {}))
        for k, v in w.get("counters", {}).items():
            snap.setdefault("counters", {}).setdefault(k, v)
    return snap


def clone_function(fn):
    """Ships a user function to a subtask the way Flink ships closures: serialize the
    descriptor (model runtime fields are transient) and deserialize a private copy."""
    return cloudpickle.loads(cloudpickle.dumps(fn))
