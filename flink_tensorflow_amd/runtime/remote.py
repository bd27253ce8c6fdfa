"""Operator subtasks in worker processes, connected by native shared-memory rings.

``DataStream.run_in_processes()`` moves every subtask of an operator into its own worker
process (``spawn``; one per GPU for model operators — ``cuda:(subtask % #GPUs)``), the
MI355X-native replacement for the TaskManager slots the reference's Flink job deploys its
subtasks to (SURVEY §2.12 "one subtask per GPU", §2.13 data exchange; the reference ships
records through ``TensorValue.write/read`` over Netty, ``LIB/types/TensorValue.java:150-187``).

Per remote subtask the coordinator keeps its usual task thread (input gates, barrier
alignment, watermarks) and forwards elements through a SPSC ring in ``/dev/shm``
(``csrc/shm_ring.cpp``) to the worker, which runs the unchanged operator (user function,
keyed state, timers, micro-batching, the GPU plan).  The worker's emissions come back on a
second ring and are re-emitted by a drainer thread in order, so a checkpoint barrier is
forwarded downstream only after every record the worker emitted before its snapshot.

Record payloads do not ride in the pickles: every ndarray / CPU tensor / ``TensorValue``
of at least ``_SLAB_MIN`` bytes is written ONCE into the edge's shared-memory tensor slab
(``TensorSlab``, a ring the coordinator allocates from) and only a descriptor (offset,
shape, dtype) crosses the ring; the worker hands the operator a zero-copy view of the slab
(e.g. the batched model operator gathers it straight into its pinned staging slot) and
returns the space when the view is garbage collected.  Small values, object payloads and a
full slab fall back to the pickle.

**Remote source chains** (``env.generate(...).run_in_processes()``): a source subtask can
run in the worker too, with the forward-connected, equal-parallelism worker operators
downstream of it chained into the same process (Flink's chained source in a task slot).
Records are then produced, mapped and consumed inside the worker — nothing crosses the
coordinator — so a parallel source feeds N model workers at the rate of N processes, not
of one coordinator thread.  Checkpoint triggers travel to the worker, which snapshots the
source offset and every chained operator between two records and sends the states and
the barrier INLINE in its output stream (ordered after everything emitted before it).

Messages (cloudpickle, fragmented when larger than half a ring):

=====================  ==============================================================
coordinator → worker   ``init`` (operator factory, context, restore state), ``recs``
                       [(value, ts, input)], ``wm`` ts, ``snap`` (id, dir), ``notify``
                       id, ``end``, ``close``; source chains: ``init_chain`` (factories,
                       contexts, restore states), ``trigger`` (id, dir), ``cancel``
worker → coordinator   ``out`` [elements], ``side`` [(tag, value)], ``state`` (id, state),
                       ``ended``, ``closed`` (metrics), ``error`` (message, traceback);
                       source chains: ``barrier`` (id, ts, [state per chain member]),
                       ``source_end`` (final source state)
=====================  ==============================================================
"""
from __future__ import annotations

import os
import queue
import threading
import time
import traceback
import uuid

import collections
import weakref

import cloudpickle
import numpy as np

from .. import _ext
from .operators import Output, Record, Watermark

_RING_BYTES = 64 << 20
_SLAB_BYTES = int(os.environ.get("FTM_SLAB_BYTES", str(1 << 30)))  # per coordinator -> worker edge
_SLAB_MIN = 4096       # payloads below this ride in the pickle
_SLAB_ALIGN = 128
_BATCH = 64
_IDLE_S = 0.02


_SLAB_TAG = "__ftm_slab_ref__"


def _SlabRef(start, pos, end, shape, dtype, kind, tv_dtype=None):  # noqa: N802
    """Descriptor of a record payload in the tensor slab (what crosses the ring): a plain
    tuple, so pickling it stays on the C fast path."""
    return (_SLAB_TAG, start, pos, end, shape, dtype, kind, tv_dtype)


def _is_ref(v) -> bool:
    return type(v) is tuple and len(v) == 8 and v[0] == _SLAB_TAG


class TensorSlab:
    """Shared-memory ring of record payloads for one coordinator -> worker edge.

    The coordinator allocates monotonically (``head``; an allocation never straddles the
    end of the ring — the rest of the ring is skipped and released with it) and copies each
    payload in once; the worker maps the same segment, hands out zero-copy numpy views and
    publishes, in the 8-byte header, the position up to which every view has been dropped
    (releases are applied in allocation order).  A full slab makes the coordinator wait
    briefly, then fall back to pickling (a window operator may legitimately hold many
    records)."""

    HDR = 64

    def __init__(self, name: str, create: bool, capacity: int = _SLAB_BYTES):
        import mmap

        self.path = "/dev/shm/" + name.lstrip("/")
        fd = os.open(self.path, (os.O_RDWR | os.O_CREAT | os.O_EXCL) if create else os.O_RDWR, 0o600)
        try:
            if create:
                os.ftruncate(fd, capacity + self.HDR)
            size = os.fstat(fd).st_size
            self._mm = mmap.mmap(fd, size, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.name = name
        self.cap = size - self.HDR
        self.mem = np.frombuffer(self._mm, np.uint8)
        self.hdr = np.frombuffer(self._mm, np.int64, 1, 0)
        self.owner = create
        self._native = _ext.native()
        self._base = self.mem.ctypes.data
        if create:
            self.hdr[0] = 0
        self.head = 0
        self.records = self.bytes = self.waits = 0
        # worker side
        self._lock = threading.Lock()
        self._pending: collections.deque = collections.deque()
        self._dropped: set = set()

    # ---- coordinator
    def reserve(self, nbytes: int, wait_s: float = 0.05):
        """Reserves ``nbytes`` contiguous bytes: (start, pos) or None (no room in time)."""
        if nbytes > self.cap // 2:
            return None
        off = self.head % self.cap
        start = self.head
        pos = self.head + (self.cap - off if off + nbytes > self.cap else 0)
        t_end = None
        while pos + nbytes - int(self.hdr[0]) > self.cap:
            self.waits += 1
            if t_end is None:
                t_end = time.time() + wait_s
            elif time.time() > t_end:
                return None
            time.sleep(1e-4)
        return start, pos

    def put_batch(self, batch: list) -> list:
        """``batch`` of (value, ts, input) with every large payload copied in (ONE native
        multithreaded scatter for the micro-batch, GIL released) and replaced by its
        descriptor; values that do not qualify, or a batch that finds no room, stay as
        they are (pickled)."""
        picks = []
        for i, (v, _ts, _ix) in enumerate(batch):
            a = _payload(v)
            if a is not None:
                picks.append((i, a))
        if not picks:
            return batch
        sizes = [-(-a[1].nbytes // _SLAB_ALIGN) * _SLAB_ALIGN for _, a in picks]
        got = self.reserve(sum(sizes))
        if got is None:
            return batch
        start, pos = got
        offs, refs, cur = [], [], pos
        out = list(batch)
        for (i, (kind, arr, tvd)), sz in zip(picks, sizes):
            offs.append(self.HDR + cur % self.cap)
            refs.append(arr)
            v, ts, ix = batch[i]
            out[i] = (_SlabRef(start if cur == pos else cur, cur, cur + sz, arr.shape, arr.dtype.str, kind, tvd),
                      ts, ix)
            cur += sz
        self._native.scatter_into(self._base, self.mem.nbytes, offs, refs, 4)
        self.head = cur
        self.records += len(picks)
        self.bytes += sum(a[1].nbytes for _, a in picks)
        return out

    # ---- worker
    def view(self, ref, track: bool = True):
        _, start, pos, end, shape, dtype, _kind, _tvd = ref
        o = self.HDR + pos % self.cap
        dt = np.dtype(dtype)
        n = int(np.prod(shape, dtype=np.int64))
        # the record's OWN base array: its base is a memoryview (not another ndarray), so
        # every view derived from the record (reshape, slices, .view(dtype)) collapses onto
        # it and keeps it alive — the release below cannot fire while any view survives
        base = np.frombuffer(memoryview(self._mm)[o:o + n * dt.itemsize], dt, n)
        with self._lock:
            self._pending.append((start, end))
        if track:
            self.track(base, start)
        return base.reshape(shape)

    def view_batch(self, refs) -> list:
        """Zero-copy arrays for the slab records of ONE ``put_batch`` (contiguous, in
        allocation order): one base array over their span, one finalizer on it, and each
        record a slice of it — so a record, and every view derived from it, keeps the batch
        base alive, and the span is released when the last of them is collected.  (Per
        record, ``frombuffer`` + a finalizer cost ~10 µs of Python: at 80k records/s a
        whole core of the worker.)"""
        first, last = refs[0], refs[-1]
        start, pos0, end = first[1], first[2], last[3]
        o0 = self.HDR + pos0 % self.cap
        base = np.frombuffer(memoryview(self._mm)[o0:o0 + (end - pos0)], np.uint8)
        with self._lock:
            self._pending.append((start, end))
        self.track(base, start)
        out = []
        for r in refs:
            pos, shape, dt = r[2], r[4], np.dtype(r[5])
            nb = dt.itemsize
            for d in shape:
                nb *= d
            a = base[pos - pos0:pos - pos0 + nb]
            out.append((a if dt == np.uint8 else a.view(dt)).reshape(shape))
        return out

    def track(self, base, start: int) -> None:
        """Releases the record's space when ``base`` (and therefore every view of it) is
        collected.  ``base`` must be the array returned by ``np.frombuffer`` in ``view``."""
        weakref.finalize(base, self._drop, start)

    def _drop(self, start):
        with self._lock:
            self._dropped.add(start)
            rel = None
            while self._pending and self._pending[0][0] in self._dropped:
                s0, e0 = self._pending.popleft()
                self._dropped.discard(s0)
                rel = e0
            if rel is not None:
                self.hdr[0] = rel

    def close(self):
        """Drops this process's mapping handle (views still alive keep the pages mapped
        until they are collected)."""
        self.mem = self.hdr = None
        self._mm = None

    def unlink(self):
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass
            self.owner = False


_TYPES: list = []


def _payload(value):
    """(kind, contiguous ndarray, TensorValue meta) of a slab-eligible record, else None."""
    if type(value) is np.ndarray:  # the common case first, no imports / isinstance chain
        if value.dtype.hasobject or value.nbytes < _SLAB_MIN:
            return None
        return "np", (value if value.flags.c_contiguous else np.ascontiguousarray(value)), None
    if not _TYPES:
        import torch

        from ..types.tensor_value import TensorValue

        _TYPES.extend((torch.Tensor, TensorValue, torch.bfloat16))
    tensor_t, tv_t, bf16 = _TYPES
    kind, arr, tvd = None, None, None
    if isinstance(value, np.ndarray):
        if not value.dtype.hasobject:
            kind, arr = "np", value
    elif isinstance(value, tensor_t):
        if value.device.type == "cpu" and value.dtype != bf16:
            kind, arr = "torch", value.detach().numpy()
    elif isinstance(value, tv_t):
        p = value._payload
        if isinstance(p, np.ndarray):
            arr = p
        elif isinstance(p, (bytes, bytearray, memoryview)):
            arr = np.frombuffer(p, np.uint8)
        if arr is not None:
            kind, tvd = "tv", (int(value.dtype), value.shape())
    if arr is None or arr.nbytes < _SLAB_MIN:
        return None
    return kind, np.ascontiguousarray(arr), tvd


def _from_slab(value, slab: TensorSlab, arr=None):
    if not _is_ref(value):
        return value
    if arr is None:
        arr = slab.view(value)
    kind = value[6]
    if kind == "torch":
        import torch

        return torch.from_numpy(arr)
    if kind == "tv":
        from ..types.tensor_value import TensorValue

        dt, shape = value[7]
        return TensorValue(dt, shape, arr)
    return arr


class RemoteTaskError(RuntimeError):
    pass


class ShmChannel:
    """One direction of a worker link: pickled messages over a ``ShmRing``."""

    def __init__(self, name: str, create: bool, capacity: int = _RING_BYTES):
        self.ring = _ext.native().ShmRing(name, capacity if create else 0, create)
        self.name = name
        self.owner = create

    def send(self, msg, timeout_s: float = -1.0, alive=None) -> int:
        data = cloudpickle.dumps(msg, protocol=5)
        step = self.ring.max_message - 1
        parts = [data[i:i + step] for i in range(0, len(data), step)] or [b""]
        for i, p in enumerate(parts):
            flag = b"\x01" if i + 1 < len(parts) else b"\x00"
            while not self.ring.push(flag + p, 0.5 if timeout_s < 0 else timeout_s):
                if alive is not None and not alive():
                    raise RemoteTaskError(f"peer of {self.name} died")
                if timeout_s >= 0:
                    raise TimeoutError(f"{self.name}: ring full")
        return len(data)

    def recv(self, timeout_s: float):
        """A message, or None on timeout (or when the producer closed the ring)."""
        chunks = []
        while True:
            m = self.ring.pop(timeout_s if not chunks else 30.0)
            if m is None:
                if chunks:
                    raise RemoteTaskError(f"{self.name}: truncated message")
                return None
            chunks.append(m[1:])
            if m[:1] == b"\x00":
                return cloudpickle.loads(b"".join(chunks))

    def close(self):
        self.ring.close_producer()

    def unlink(self):
        if self.owner:
            _ext.native().ShmRing.unlink(self.name)
            self.owner = False


# ------------------------------------------------------------------ worker side
def _open_group(spec, device):
    """Joins the operator's communicator (``LocalExecutor.operator_group``): RCCL on the
    subtask's GPU, or the test implementation the job injected.  It is bound to THIS
    operator's calls (``_GroupBound``), not installed process-wide: two grouped operators
    chained in one worker each keep their own group."""
    g = spec.get("group")
    if not g:
        return None
    import datetime

    from torch.distributed import PrefixStore, TCPStore

    from ..parallel import comm

    if not g.get("cls") and (device is None or device.type != "cuda"):
        return None
    store = PrefixStore(g["prefix"], TCPStore(g["addr"], g["port"], g["size"], is_master=False,
                                              timeout=datetime.timedelta(seconds=600)))
    if g.get("cls"):
        c = cloudpickle.loads(g["cls"])(spec["subtask"], g["size"], device or "cpu", store)
    else:
        c = comm.RcclCommunicator(spec["subtask"], g["size"], device, store)
    return c


def _close_group(c, abort: bool) -> None:
    if c is None:
        return
    try:
        c.destroy(abort=abort)  # a failed subtask aborts: the restarted attempt builds a new group
    except Exception:  # noqa: BLE001
        pass


class _GroupBound:
    """An operator whose every call runs with its communicator bound
    (``parallel.comm.bound``): ``comm.get()`` / ``is_dist()`` inside the operator — model
    open, broadcasts, collective training steps, snapshots — see this operator's group,
    whichever thread makes the call (task loop, chain timer)."""

    _CALLS = ("setup", "initialize", "open", "close", "process", "process_batch", "process_many", "process_watermark",
              "on_idle", "next_deadline", "end_input", "prepare_snapshot", "snapshot_state",
              "notify_checkpoint_complete")

    def __init__(self, op, group):
        self.__dict__["_op"], self.__dict__["_group"] = op, group
        self.__dict__["_calls"] = {}

    def __getattr__(self, name):
        a = getattr(self._op, name)
        if name not in self._CALLS or self._group is None:
            return a
        c = self._calls.get(name)
        if c is not None and c[0] is a:
            return c[1]
        from ..parallel.comm import _BOUND

        group = self._group

        def call(*args, **kw):  # the per-record path: a plain context-variable set / reset
            tok = _BOUND.set(group)
            try:
                return a(*args, **kw)
            finally:
                _BOUND.reset(tok)
        self._calls[name] = (a, call)
        return call

    def __setattr__(self, name, value):
        setattr(self._op, name, value)


def _worker_main(in_name: str, out_name: str, slab_name: str | None = None):
    inp = ShmChannel(in_name, create=False)
    out = ShmChannel(out_name, create=False)
    slab = TensorSlab(slab_name, create=False) if slab_name else None
    op = None
    group = None
    profiler = None
    pending: list = []
    parent = os.getppid()

    def parent_alive() -> bool:
        return os.getppid() == parent

    def flush():
        if pending:
            out.send(("out", list(pending)), alive=parent_alive)  # a full ring never outlives the coordinator
            pending.clear()

    def emit(elem):
        pending.append(elem)
        if len(pending) >= _BATCH or not isinstance(elem, Record):
            flush()

    try:
        out.send(("attached",))  # the coordinator may now unlink the segment names
        while True:
            msg = inp.recv(1.0)
            if msg is not None:
                break
            if not parent_alive():
                return  # coordinator gone
        if msg[0] == "init_chain":
            prof = os.environ.get("FTM_WORKER_PROFILE")  # diagnostics: cProfile of the chain's thread
            if prof:
                import cProfile

                pr = cProfile.Profile()
                try:
                    pr.runcall(_run_source_chain, msg, inp, out, emit, flush, parent_alive)
                finally:
                    pr.dump_stats(f"{prof}.{os.getpid()}")
            else:
                _run_source_chain(msg, inp, out, emit, flush, parent_alive)
            op = None
            return
        kind, factory, spec, restore, restore_dir = msg
        assert kind == "init", kind
        from .functions import RuntimeContext
        from ..utils.metrics import MetricGroup

        device = _worker_device(spec)
        if os.environ.get("FTM_WORKER_PROFILE"):  # diagnostics: cProfile of the operator loop
            import cProfile

            profiler = cProfile.Profile()
            profiler.enable()
        metrics = MetricGroup(f"{spec['name']}[{spec['subtask']}]")
        ctx = RuntimeContext(spec["name"], spec["subtask"], spec["parallelism"], device, spec["attempt"], metrics,
                             spec["config"], None)
        ctx.global_index, ctx.global_parallelism = spec["global_index"], spec["global_parallelism"]
        ctx.restart_attempts = spec.get("restarts")
        ctx.worker_pid = os.getpid()
        group = _open_group(spec, device)
        op = _GroupBound(cloudpickle.loads(factory)(), group)
        op.setup(ctx, Output(emit, lambda tag, v: (flush(), out.send(("side", [(tag, v)]), alive=parent_alive))))
        op.initialize(restore, restore_dir)
        op.open()
        while True:
            msg = inp.recv(_IDLE_S)
            if msg is None:
                if not parent_alive():
                    break  # orphaned: the coordinator died
                op.on_idle(time.time())
                flush()
                continue
            kind = msg[0]
            if kind == "recs":
                items = msg[1]
                arrs = None
                if slab is not None:
                    # the message's slab records (one put_batch) as slices of one base array:
                    # released when the last view of any of them is collected — at once when
                    # the operator kept nothing (maps, batch staging copies), later when it
                    # kept a record or a view derived from one (windows, keyed state, pending
                    # micro-batches)
                    refs = [v for v, _, _ in items if _is_ref(v)]
                    if refs:
                        arrs = iter(slab.view_batch(refs))
                batch_fn = getattr(op, "process_batch", None) if arrs is None and items else None
                if batch_fn is not None and all(it[2] == items[0][2] for it in items):
                    # a plain run from one input: one call (the chained file reader reads the
                    # run's files in one native call and hands the model one run)
                    batch_fn([Record(v, ts) for v, ts, _ in items], items[0][2])
                else:
                    for value, ts, idx in items:
                        if arrs is not None and _is_ref(value):
                            a = next(arrs)
                            value = a if value[6] == "np" else _from_slab(value, slab, a)
                        op.process(Record(value, ts), idx)
                metrics.inc("records_in", len(items))
            elif kind == "wm":
                op.process_watermark(Watermark(msg[1]))
            elif kind == "snap":
                op.prepare_snapshot()
                state = op.snapshot_state(msg[1], msg[2])
                flush()
                out.send(("state", msg[1], state), alive=parent_alive)
                continue
            elif kind == "notify":
                op.notify_checkpoint_complete(msg[1])
            elif kind == "end":
                op.end_input()
                flush()
                out.send(("ended",), alive=parent_alive)
                continue
            elif kind == "close":
                op.close()
                op = None
                _close_group(group, abort=False)
                group = None
                if profiler is not None:  # before "closed": the coordinator may reap us after it
                    profiler.disable()
                    profiler.dump_stats(f"{os.environ['FTM_WORKER_PROFILE']}.{os.getpid()}")
                    profiler = None
                flush()
                out.send(("closed", metrics.snapshot()), alive=parent_alive)
                break
            op.on_idle(time.time())
            flush()
    except BaseException as e:  # noqa: BLE001
        try:
            pending.clear()
            out.send(("error", f"{type(e).__name__}: {e}", traceback.format_exc()), timeout_s=5.0)
        except Exception:  # noqa: BLE001
            pass
    finally:
        if op is not None:
            try:
                op.close()
            except Exception:  # noqa: BLE001
                pass
        _close_group(group, abort=True)
        if profiler is not None:
            profiler.disable()
            profiler.dump_stats(f"{os.environ['FTM_WORKER_PROFILE']}.{os.getpid()}")
        out.close()



class _ChainCancelled(Exception):
    pass


def _worker_device(spec):
    if not spec["gpu"]:
        return None
    import torch

    if not torch.cuda.is_available():
        return None
    from ..parallel.comm import gpu_count

    device = torch.device("cuda", spec["subtask"] % max(1, gpu_count()))
    torch.cuda.set_device(device)
    if os.environ.get("FT_NUMA_BIND", "1") != "0":
        from ..parallel.comm import bind_to_gpu_numa

        # the subtask's host staging (gather / decode pools started after this) runs on its
        # GPU's socket, as the SPMD ranks do (bench.py)
        bind_to_gpu_numa(device)
    return device


def _run_source_chain(msg, inp, out, emit, flush, parent_alive):
    """Worker side of a remote source chain: the source function runs here and every record
    goes straight through the chained operators; only the chain's output leaves."""
    from .functions import RuntimeContext, SourceContext
    from ..utils.metrics import MetricGroup

    _, factories, specs, restores, restore_dir = msg
    ops = [cloudpickle.loads(f)() for f in factories]
    metrics = []
    # the source node itself never uses the GPU: bind the device of the first GPU member
    gpu_spec = next((sp for sp in specs if sp["gpu"]), None)
    device = _worker_device(gpu_spec) if gpu_spec is not None else None

    def side(tag, v):
        flush()
        out.send(("side", [(tag, v)]), alive=parent_alive)

    def into(nxt):
        def e(elem):
            if type(elem) is Record:
                nxt.process(elem, 0)  # (_GroupBound caches the bound call: no per-record closure)
            elif isinstance(elem, Watermark):
                nxt.process_watermark(elem, 0)
            else:
                raise TypeError(f"operators emit records and watermarks, not {type(elem).__name__}")
        return e

    # one communicator per grouped member, bound to that member's calls
    groups = [_open_group(sp, device) if sp["gpu"] else None for sp in specs]
    ops = [_GroupBound(o, g) for o, g in zip(ops, groups)]
    for i, (op, sp) in enumerate(zip(ops, specs)):
        mg = MetricGroup(f"{sp['name']}[{sp['subtask']}]")
        metrics.append(mg)
        ctx = RuntimeContext(sp["name"], sp["subtask"], sp["parallelism"], device if sp["gpu"] else None,
                             sp["attempt"], mg, sp["config"], None)
        ctx.global_index, ctx.global_parallelism = sp["global_index"], sp["global_parallelism"]
        ctx.restart_attempts = sp.get("restarts")
        ctx.worker_pid = os.getpid()
        op.setup(ctx, Output(into(ops[i + 1]) if i + 1 < len(ops) else emit, side))
        op.initialize(restores[i], restore_dir)
    for op in reversed(ops):
        op.open()
    head = into(ops[1]) if len(ops) > 1 else emit
    bulk_head = getattr(ops[1], "process_many", None) if len(ops) > 1 else None
    src, fn = ops[0], ops[0].fn
    lock = threading.RLock()
    last = [time.perf_counter()]
    recs_out = [0]

    def control(m):
        kind = m[0]
        if kind == "trigger":
            cid, d = m[1], m[2]
            with lock:
                for o in ops[1:]:
                    o.prepare_snapshot()
                states = [o.snapshot_state(cid, d) for o in ops]
                flush()
                out.send(("barrier", cid, time.time(), states), alive=parent_alive)
        elif kind == "notify":
            for o in ops:
                o.notify_checkpoint_complete(m[1])
        elif kind == "cancel":
            fn.cancel()
            raise _ChainCancelled()
        else:
            raise RemoteTaskError(f"unexpected {kind!r} while the source runs")

    def poll(force=False):
        now = time.perf_counter()
        if not force and now - last[0] < 1e-3:
            return
        last[0] = now
        while True:
            m = inp.recv(0.0)
            if m is None:
                break
            control(m)
        if not parent_alive():
            raise _ChainCancelled()
        for o in ops[1:]:
            o.on_idle(time.time())
        flush()

    class Ctx(SourceContext):
        @property
        def checkpoint_lock(self):
            return lock

        def collect(self, value, timestamp=None):
            with lock:  # re-entrant: sources normally hold it already (chain timer excluded)
                poll()
                head(Record(value, timestamp))
            recs_out[0] += 1

        def collect_many(self, values, timestamp=None):
            with lock:
                poll()
                if bulk_head is not None:  # a micro-batching first member takes the run at once
                    bulk_head(values, timestamp)
                else:
                    for v in values:
                        head(Record(v, timestamp))
            recs_out[0] += len(values)

        def emit_watermark(self, ts):
            with lock:
                head(Watermark(ts))

    stop = threading.Event()
    timer_error: list = []

    def chain_timer():
        # the local chain's ``_chain_timer`` (executor.py): while the source blocks between
        # records (slow generator, file-monitor sleep) the chained operators still get their
        # deadlines (micro-batch max_delay, completed GPU batches) and checkpoint triggers
        # still get their barrier; the collect path polls while records flow
        try:
            while True:
                with lock:
                    dls = [d for d in (o.next_deadline() for o in ops[1:]) if d is not None]
                wait = 0.01 if not dls else min(0.01, max(2e-4, min(dls) - time.time()))
                if stop.wait(wait):
                    return
                if time.perf_counter() - last[0] < wait:
                    continue  # the source is emitting: the collect path polls
                with lock:
                    if stop.is_set():
                        return
                    poll(force=True)
        except BaseException as e:  # noqa: BLE001 - _ChainCancelled included: re-raised after the source returns
            timer_error.append(e)
            fn.cancel()

    timer = threading.Thread(target=chain_timer, name="worker-chain-timer", daemon=True)
    timer.start()
    try:
        try:
            fn.run(Ctx())
        finally:
            with lock:
                stop.set()
            timer.join()
        if timer_error:
            raise timer_error[0]
        with lock:
            poll(force=True)  # triggers that arrived before the end still get their barrier
            final = src.snapshot_state(-1, None)
        head(Watermark(float("inf")))
        for o in ops[1:]:
            o.end_input()
        flush()
        out.send(("source_end", final), alive=parent_alive)
        while True:  # late notifications, then close
            m = inp.recv(_IDLE_S)
            if m is None:
                if not parent_alive():
                    return
                continue
            if m[0] == "notify":
                for o in ops:
                    o.notify_checkpoint_complete(m[1])
            elif m[0] == "close":
                break
            elif m[0] == "cancel":
                return
        for o in ops:
            o.close()
        ops = []
        for g in groups:
            _close_group(g, abort=False)
        groups = []
        metrics[0].inc("records_out", recs_out[0])
        out.send(("closed", [mg.snapshot() for mg in metrics]), alive=parent_alive)
    except _ChainCancelled:
        pass
    finally:
        for o in ops:
            try:
                o.close()
            except Exception:  # noqa: BLE001
                pass
        for g in groups:
            _close_group(g, abort=True)

# ------------------------------------------------------------------ coordinator side
def _job_group(job, node):
    f = getattr(job, "operator_group", None)
    return f(node) if f is not None and getattr(node, "uses_gpu", False) else None


# (operator name, subtask) -> the last attempt's coordinator -> worker record traffic
TRANSPORT_STATS: dict = {}


class RemoteOperatorProxy:
    """Stands in for the operator inside the coordinator's task loop."""

    chainable = False

    def __init__(self, node, subtask: int, job, ring_bytes: int = _RING_BYTES):
        self.node = node
        self.subtask = subtask
        self.job = job
        self.num_inputs = 1
        self.ring_bytes = ring_bytes
        self.to_worker = self.from_worker = None  # created when the subtask starts
        self.slab: TensorSlab | None = None
        self.proc = None
        self.out: Output | None = None
        self.ctx = None
        self._buf: list = []
        self._replies: queue.Queue = queue.Queue()
        self._send_lock = threading.Lock()
        self._error: tuple | None = None
        self._drainer: threading.Thread | None = None
        self.worker_metrics: dict | None = None
        # coordinator -> worker record traffic: records, bytes of the "recs" messages on the
        # ring (pickled values or slab descriptors) and payload bytes through the slab
        self.stats = {"records": 0, "ring_bytes": 0, "slab_bytes": 0}

    # ---- lifecycle (called by the task thread)
    def setup(self, ctx, out: Output):
        self.ctx = ctx
        self.out = out

    def initialize(self, snapshot, checkpoint_dir):
        try:
            self._start(snapshot, checkpoint_dir)
        except BaseException:
            self._shutdown()
            raise

    def _start(self, snapshot, checkpoint_dir):
        import multiprocessing as mp

        tag = f"/ftm-{os.getpid()}-{uuid.uuid4().hex[:10]}"
        self.to_worker = ShmChannel(tag + "-in", True, self.ring_bytes)
        self.from_worker = ShmChannel(tag + "-out", True, self.ring_bytes)
        self.slab = TensorSlab(tag + "-slab", True, _SLAB_BYTES) if _SLAB_BYTES > 0 else None
        self.proc = mp.get_context("spawn").Process(target=_worker_main, name=f"ftm-{self.node.name}-{self.subtask}",
                                                    args=(self.to_worker.name, self.from_worker.name,
                                                          self.slab.name if self.slab else None), daemon=True)
        self.proc.start()
        self._drainer = threading.Thread(target=self._drain, name=f"drain-{self.node.name}-{self.subtask}",
                                         daemon=True)
        self._drainer.start()
        self._wait("attached", 120.0)
        self.to_worker.unlink()  # both ends are mapped: the names can go (no /dev/shm leak on a crash)
        self.from_worker.unlink()
        if self.slab is not None:
            self.slab.unlink()
        spec = {"name": self.node.name, "subtask": self.subtask, "parallelism": self.node.parallelism,
                "gpu": bool(self.node.uses_gpu), "attempt": self.job.attempt, "config": self.job.config,
                "restarts": self.job.env.restart_strategy.attempts,
                "global_index": self.ctx.global_index, "global_parallelism": self.ctx.global_parallelism,
                "group": _job_group(self.job, self.node)}
        self._send(("init", cloudpickle.dumps(self.node.factory), spec, snapshot, checkpoint_dir))

    def open(self):
        pass

    def close(self):
        graceful = False
        try:
            if self._alive() and self._error is None and not self.job.cancel.is_set():
                self._flush()
                self._send(("close",))
                self._wait("closed", 60.0)
                graceful = True
        finally:
            self._shutdown(graceful)

    def _shutdown(self, graceful: bool = False):
        TRANSPORT_STATS[(self.node.name, self.subtask)] = dict(self.stats)
        if self.proc is not None:
            if not graceful and self.proc.is_alive():
                self.proc.terminate()  # failed / cancelled attempt: its state is discarded anyway
            self.proc.join(timeout=10)
            if self.proc.is_alive():
                self.proc.kill()
                self.proc.join(timeout=5)
        if self.from_worker is not None:
            self.from_worker.close()  # wakes the drainer if it is still waiting
        if self._drainer is not None:
            self._drainer.join(timeout=5)
        for ch in (self.to_worker, self.from_worker):
            if ch is not None:
                ch.unlink()
        if self.slab is not None:
            if os.environ.get("FTM_SLAB_DEBUG"):
                print(f"[slab] {self.node.name}[{self.subtask}] records={self.slab.records} "
                      f"bytes={self.slab.bytes} waits={self.slab.waits} head={self.slab.head}", flush=True)
            self.slab.unlink()
            self.slab.close()
            self.slab = None

    # ---- data path
    def process(self, rec: Record, input_index: int = 0):
        self._buf.append((rec.value, rec.ts, input_index))
        if len(self._buf) >= _BATCH:
            self._flush()

    def process_watermark(self, wm: Watermark, input_index: int = 0):
        self._flush()
        self._send(("wm", wm.ts))

    def on_idle(self, now: float):
        self._flush()
        self._check()

    def next_deadline(self):
        return None  # the worker runs its own timers between messages

    def end_input(self):
        self._flush()
        self._send(("end",))
        self._wait("ended", None)

    # ---- checkpoints
    def prepare_snapshot(self):
        self._flush()

    def snapshot_state(self, checkpoint_id: int, checkpoint_dir):
        self._send(("snap", checkpoint_id, checkpoint_dir))
        return self._wait("state", None)[2]

    def notify_checkpoint_complete(self, checkpoint_id: int):
        self._send(("notify", checkpoint_id))

    def _on_barrier(self, msg):
        raise RemoteTaskError(f"{self.node.name}[{self.subtask}]: unexpected barrier from an operator worker")

    # ---- plumbing
    def _alive(self) -> bool:
        return self.proc is not None and self.proc.is_alive()

    def _send(self, msg) -> int:
        self._check()
        with self._send_lock:  # task thread + checkpoint-complete notifications: one producer at a time
            return self.to_worker.send(msg, alive=self._alive)

    def _flush(self):
        if self._buf:
            batch, self._buf = self._buf, []
            if self.slab is not None:
                b0 = self.slab.bytes
                batch = self.slab.put_batch(batch)
                self.stats["slab_bytes"] += self.slab.bytes - b0
            self.stats["records"] += len(batch)
            self.stats["ring_bytes"] += self._send(("recs", batch))

    def _check(self):
        if self._error is not None:
            raise RemoteTaskError(f"{self.node.name}[{self.subtask}] worker failed: {self._error[0]}\n{self._error[1]}")

    def _wait(self, kind: str, timeout_s):
        t_end = None if timeout_s is None else time.time() + timeout_s
        while True:
            self._check()
            try:
                msg = self._replies.get(timeout=0.1)
            except queue.Empty:
                if t_end is not None and time.time() > t_end:
                    raise TimeoutError(f"{self.node.name}[{self.subtask}]: no {kind!r} from the worker") from None
                if self.job.cancel.is_set():
                    from .executor import JobCancelled

                    raise JobCancelled() from None
                continue
            if msg[0] != kind:
                raise RemoteTaskError(f"{self.node.name}[{self.subtask}]: expected {kind!r}, got {msg[0]!r}")
            return msg

    def _drain(self):
        """Re-emits the worker's output in order; hands control replies to the task."""
        while True:
            try:
                msg = self.from_worker.recv(0.2)
            except Exception as e:  # noqa: BLE001
                self._error = (f"{type(e).__name__}: {e}", traceback.format_exc())
                return
            if msg is None:
                if self.from_worker.ring.closed and self.from_worker.ring.used == 0:
                    if self._error is None and self.worker_metrics is None:
                        self._error = ("worker exited without closing", "")
                    return
                if self.proc is not None and not self.proc.is_alive() and self.from_worker.ring.used == 0:
                    if self.worker_metrics is None and self._error is None:
                        self._error = (f"worker process died (exit code {self.proc.exitcode})", "")
                    return
                continue
            kind = msg[0]
            try:
                if kind == "out":
                    for elem in msg[1]:
                        self.out._emit(elem)
                elif kind == "side":
                    for tag, v in msg[1]:
                        self.out.emit_side(tag, v)
                elif kind == "error":
                    self._error = (msg[1], msg[2])
                    return
                elif kind == "barrier":
                    self._on_barrier(msg)
                else:
                    if kind == "closed":
                        self.worker_metrics = msg[1]
                    self._replies.put(msg)
                    if kind == "closed":
                        return
            except Exception as e:  # noqa: BLE001 - e.g. a cancelled downstream
                self._error = (f"{type(e).__name__}: {e}", traceback.format_exc())
                return


class RemoteChainProxy(RemoteOperatorProxy):
    """Coordinator side of a remote source chain (``nodes[0]`` the source, then the chained
    worker operators).  The drainer re-emits the chain's output, acknowledges each member's
    snapshot and forwards the barrier when the worker's inline ``barrier`` message arrives."""

    def __init__(self, nodes, subtask: int, job, ring_bytes: int = _RING_BYTES):
        super().__init__(nodes[0], subtask, job, ring_bytes)
        self.nodes = list(nodes)
        self.final_state = None

    def start_chain(self, contexts, restores, checkpoint_dir):
        try:
            self._start_chain(contexts, restores, checkpoint_dir)
        except BaseException:
            self._shutdown()
            raise

    def _start_chain(self, contexts, restores, checkpoint_dir):
        import multiprocessing as mp

        tag = f"/ftm-{os.getpid()}-{uuid.uuid4().hex[:10]}"
        self.to_worker = ShmChannel(tag + "-in", True, self.ring_bytes)
        self.from_worker = ShmChannel(tag + "-out", True, self.ring_bytes)
        name = "+".join(n.name for n in self.nodes)
        self.proc = mp.get_context("spawn").Process(target=_worker_main, name=f"ftm-{name}-{self.subtask}",
                                                    args=(self.to_worker.name, self.from_worker.name, None),
                                                    daemon=True)
        self.proc.start()
        self._drainer = threading.Thread(target=self._drain, name=f"drain-{name}-{self.subtask}", daemon=True)
        self._drainer.start()
        self._wait("attached", 120.0)
        self.to_worker.unlink()
        self.from_worker.unlink()
        specs = [{"name": n.name, "subtask": self.subtask, "parallelism": n.parallelism, "gpu": bool(n.uses_gpu),
                  "attempt": self.job.attempt, "config": self.job.config, "global_index": c.global_index,
                  "restarts": self.job.env.restart_strategy.attempts,
                  "global_parallelism": c.global_parallelism, "group": _job_group(self.job, n)}
                 for n, c in zip(self.nodes, contexts)]
        self._send(("init_chain", [cloudpickle.dumps(n.factory) for n in self.nodes], specs, list(restores),
                    checkpoint_dir))

    def trigger(self, checkpoint_id: int, checkpoint_dir):
        self._send(("trigger", checkpoint_id, checkpoint_dir))

    def cancel(self):
        if self._alive():
            try:
                self.to_worker.send(("cancel",), timeout_s=1.0)
            except Exception:  # noqa: BLE001
                pass

    def wait_source_end(self, cancel) -> object:
        """Blocks until the worker's source finished (its final state), raising on a worker
        failure or a cancelled job; ``cancel()`` is polled between waits."""
        while True:
            self._check()
            try:
                msg = self._replies.get(timeout=0.05)
            except queue.Empty:
                cancel()
                continue
            if msg[0] != "source_end":
                raise RemoteTaskError(f"{self.node.name}[{self.subtask}]: expected 'source_end', got {msg[0]!r}")
            self.final_state = msg[1]
            return msg[1]

    def close(self):
        graceful = False
        try:
            if self._alive() and self._error is None and not self.job.cancel.is_set():
                self._send(("close",))
                self._wait("closed", 60.0)
                graceful = True
        finally:
            self._shutdown(graceful)

    def _drain(self):
        super()._drain()
        m = self.worker_metrics  # the chain sends one snapshot per member: the source's is the proxy's
        if isinstance(m, list):
            self.member_metrics = m[1:]
            self.worker_metrics = m[0] if m else None

    def _on_barrier(self, msg):
        from .operators import Barrier

        _, cid, ts, states = msg
        for n, st in zip(self.nodes, states):
            self.job.ack(cid, (n.uid, self.subtask), st)
        self.out._emit(Barrier(cid, ts))
