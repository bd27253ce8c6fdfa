"""Collectives for data-parallel inference and online training.

One process per GPU, one **RCCL communicator** per job, driven directly through the RCCL
C API (``csrc_rccl/rccl.cpp`` → ``_rccl``) — no torch.distributed process group and no
backend switch:

* **rendezvous** — rank 0 calls ``ncclGetUniqueId`` and publishes the 128 bytes in the
  launcher's key/value store (our launcher's TCP store, or torchrun's agent store when run
  under ``torch.distributed.run``); every rank then calls ``ncclCommInitRank`` on its GPU;
* **collectives** are enqueued on HIP streams on the tensors' device memory (no host
  staging): synchronous calls run on the caller's current stream, ``*_async`` calls on a
  dedicated communication stream ordered after the caller's work, returning a
  :class:`Work` whose ``wait()`` makes the caller's stream wait (overlap with compute);
* **restart** — ``destroy(abort=True)`` aborts the communicator without waiting for dead
  peers; a relaunched group rendezvouses under a fresh attempt prefix.

Framework call sites (SURVEY §2.13 "collectives call sites"):

* ``broadcast_tensors`` — rank 0 loads / compiles the model, every other rank receives
  the weights.  Large contiguous tensors are broadcast in place; small ones are packed
  into ONE fixed-size staging bucket per dtype (bounded extra HBM, not a full-model
  ``torch.cat`` copy); all calls of a round are fused in one RCCL group so the root drives
  its 7 xGMI links concurrently;
* ``GradBucketer`` — bucketed gradient all-reduce for online training, launched from
  autograd hooks as buckets fill so communication overlaps backward on the comm stream
  (bucket size chosen for per-link-bound rings on point-to-point xGMI, default 25 MB);
* ``barrier`` / ``all_reduce_scalar`` / ``all_gather_object`` / ``allgather_metrics`` —
  checkpoint alignment and whole-node metrics (latency percentiles, records/s).

CPU multi-process tests inject the test-only loopback communicator
(``parallel/fake.py``) through ``init_distributed(communicator=FakeCommunicator)``; the
product path never selects it.
"""
from __future__ import annotations

import abc
import contextlib
import contextvars
import datetime
import os
import pickle
from typing import Iterable, Sequence

import numpy as np
import torch

# RCCL datatype codes (rccl.h ncclDataType_t) and reduction codes (ncclRedOp_t)
_NCCL_DTYPE = {torch.int8: 0, torch.uint8: 1, torch.bool: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6,
               torch.float32: 7, torch.float64: 8, torch.bfloat16: 9, torch.float8_e4m3fn: 10,
               torch.float8_e5m2: 11}
_NCCL_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}

BROADCAST_BUCKET_BYTES = 64 << 20  # staging bucket for small tensors (per dtype, reused)


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the launcher environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def gpu_count() -> int:
    """Visible GPUs.  ``torch.cuda.device_count()`` may answer 0 from its non-initialising
    probe on a box where the HIP runtime does see the card; ask the runtime then."""
    n = torch.cuda.device_count()
    if n == 0 and torch.cuda.is_available():
        n = torch._C._cuda_getDeviceCount()
    return n


def local_device(local_rank: int) -> int:
    """GPU index of a local rank (wraps when ranks outnumber visible GPUs — rehearsal only)."""
    n = torch.cuda.device_count()
    return local_rank % n if n else 0


def _cpulist(text: str) -> set[int]:
    out = set()
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def bind_to_gpu_numa(device) -> dict | None:
    """Pins this rank's CPU threads to the NUMA node of its GPU (best effort).

    Every DP rank stages ~10 GB/s of decoded records through pinned host memory on an
    8-GPU node; threads started after this call (the C++ gather pool) inherit the mask and
    first-touch their staging memory on the GPU's socket instead of across the
    inter-socket link.  Returns ``{"numa_node", "cpus"}`` or None when nothing was changed
    (no NUMA info, or the allowed CPUs are all on another node)."""
    try:
        p = torch.cuda.get_device_properties(device)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as f:
            node = int(f.read())
        if node < 0:
            return None
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            cpus = _cpulist(f.read())
        allowed = os.sched_getaffinity(0)
        mine = cpus & allowed
        if not mine or mine == allowed:
            return None
        os.sched_setaffinity(0, mine)
        return {"numa_node": node, "cpus": len(mine)}
    except (OSError, ValueError, AttributeError, RuntimeError):
        return None


# ---------------------------------------------------------------------------- rendezvous
def rendezvous_store(rank: int, ws: int, timeout_s: int = 600):
    """The job's key/value store: torchrun's agent store when launched by
    ``torch.distributed.run`` (it already listens on MASTER_PORT), else a TCP store hosted
    by rank 0.  Keys live under ``ftm/<attempt>/`` so a restarted group never reads a
    previous attempt's unique id."""
    from torch.distributed import PrefixStore, TCPStore

    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29511"))
    td = datetime.timedelta(seconds=timeout_s)
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
        store = TCPStore(host, port, ws, is_master=False, timeout=td)
    else:
        store = TCPStore(host, port, ws, is_master=(rank == 0), timeout=td)
    attempt = os.environ.get("FTM_ATTEMPT", os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    return PrefixStore(f"ftm/{attempt}/", store)


# ---------------------------------------------------------------------------- communicators
class Work:
    """Handle of an asynchronous collective."""

    def __init__(self, event=None, device=None):
        self._event = event
        self._device = device

    def wait(self) -> None:
        """Orders the caller's current stream after the collective (no host sync)."""
        if self._event is not None:
            torch.cuda.current_stream(self._device).wait_event(self._event)


class Communicator(abc.ABC):
    """Collectives over one group of ranks (in place on ``tensor``; contiguous tensors)."""

    rank: int
    size: int
    device: torch.device

    @abc.abstractmethod
    def broadcast(self, t: torch.Tensor, root: int = 0) -> None: ...

    @abc.abstractmethod
    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> None: ...

    @abc.abstractmethod
    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        """``out`` holds ``size`` concatenated copies of ``inp``'s shape (rank order)."""

    @abc.abstractmethod
    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> None: ...

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum") -> Work:
        self.all_reduce(t, op)
        return Work()

    def all_to_all_v(self, out: torch.Tensor, out_splits: Sequence[int], inp: torch.Tensor,
                     in_splits: Sequence[int]) -> None:
        """Personalised exchange along dim 0: rows ``in_splits[r]`` of ``inp`` (in rank
        order) go to rank r; ``out`` receives ``out_splits[r]`` rows from rank r, in rank
        order.  The splits are host integers every pair agrees on."""
        raise NotImplementedError

    def group(self):
        """Context manager fusing the collectives issued inside into one launch."""
        import contextlib

        return contextlib.nullcontext()

    def all_gather_object(self, obj) -> list:
        data = np.frombuffer(pickle.dumps(obj), np.uint8)
        dev = self.device
        n = torch.tensor([data.size], dtype=torch.int64, device=dev)
        sizes = torch.empty(self.size, dtype=torch.int64, device=dev)
        self.all_gather(sizes, n)
        sizes = sizes.cpu().tolist()
        cap = max(sizes)
        buf = torch.zeros(cap, dtype=torch.uint8)
        buf[:data.size] = torch.from_numpy(data.copy())
        buf = buf.to(dev)
        out = torch.empty(self.size * cap, dtype=torch.uint8, device=dev)
        self.all_gather(out, buf)
        host = out.cpu().numpy()
        return [pickle.loads(host[r * cap:r * cap + sizes[r]].tobytes()) for r in range(self.size)]

    def barrier(self) -> None:
        t = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.all_reduce(t)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def destroy(self, abort: bool = False) -> None:  # noqa: B027 - optional hook
        pass


def _check(t: torch.Tensor, dev: torch.device) -> None:
    if t.device != dev:
        raise ValueError(f"collective tensor on {t.device}, communicator on {dev}")
    if not t.is_contiguous():
        raise ValueError("collective tensors must be contiguous")


class RcclCommunicator(Communicator):
    """RCCL communicator bound to this rank's GPU (``_rccl.Comm``)."""

    def __init__(self, rank: int, size: int, device, store=None, unique_id: bytes | None = None):
        from .. import _ext

        self._lib = _ext.rccl()
        self.rank, self.size = rank, size
        self.store = store  # the rendezvous store: also the host control channel (step agreement)
        self.device = torch.device(device)
        if unique_id is None:
            if rank == 0:
                unique_id = self._lib.unique_id()
                if store is not None:
                    store.set("rccl_unique_id", unique_id)
            else:
                unique_id = store.get("rccl_unique_id")
        torch.cuda.set_device(self.device)
        self._c = self._lib.Comm(unique_id, size, rank, self.device.index)
        self._stream = torch.cuda.Stream(self.device)  # async collectives (overlap with backward)

    def _dt(self, t):
        try:
            return _NCCL_DTYPE[t.dtype]
        except KeyError:
            raise TypeError(f"RCCL has no datatype for {t.dtype}") from None

    def _cur(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def broadcast(self, t, root=0):
        _check(t, self.device)
        self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), root, self._cur())

    def all_reduce(self, t, op="sum"):
        _check(t, self.device)
        self._c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), _NCCL_OP[op], self._cur())

    def all_gather(self, out, inp):
        _check(out, self.device)
        _check(inp, self.device)
        if out.numel() != inp.numel() * self.size or out.dtype != inp.dtype:
            raise ValueError("all_gather: out must hold size x inp elements of inp's dtype")
        self._c.all_gather(inp.data_ptr(), out.data_ptr(), inp.numel(), self._dt(inp), self._cur())

    def reduce_scatter(self, out, inp, op="sum"):
        _check(out, self.device)
        _check(inp, self.device)
        if inp.numel() != out.numel() * self.size or out.dtype != inp.dtype:
            raise ValueError("reduce_scatter: inp must hold size x out elements of out's dtype")
        self._c.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), self._dt(out), _NCCL_OP[op],
                               self._cur())

    def all_to_all_v(self, out, out_splits, inp, in_splits):
        _check(out, self.device)
        _check(inp, self.device)
        row = int(np.prod(inp.shape[1:])) if inp.dim() > 1 else 1
        dt, st = self._dt(inp), self._cur()
        esz = inp.element_size()
        with self.group():  # one send + one recv per peer, one launch
            o = 0
            for r, n in enumerate(in_splits):
                if n:
                    self._c.send(inp.data_ptr() + o * row * esz, n * row, dt, r, st)
                o += n
            o = 0
            for r, n in enumerate(out_splits):
                if n:
                    self._c.recv(out.data_ptr() + o * row * esz, n * row, dt, r, st)
                o += n

    def all_reduce_async(self, t, op="sum") -> Work:
        _check(t, self.device)
        s = self._stream
        s.wait_stream(torch.cuda.current_stream(self.device))  # after the producer of ``t``
        self._c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), _NCCL_OP[op], s.cuda_stream)
        t.record_stream(s)
        ev = torch.cuda.Event()
        ev.record(s)
        return Work(ev, self.device)

    def group(self):
        lib = self._lib

        class _G:
            def __enter__(self_):
                lib.group_start()

            def __exit__(self_, *a):
                lib.group_end()

        return _G()

    def async_error(self) -> str:
        return self._c.async_error()

    def destroy(self, abort=False):
        if abort:
            self._c.abort()
        else:
            self._c.destroy()


_COMM: Communicator | None = None
# one communicator per OPERATOR: a worker process running several grouped GPU operators
# (a chain) binds each operator's group around that operator's calls (``bound``); the
# process-wide ``_COMM`` (SPMD launch) is the fallback
_BOUND: contextvars.ContextVar = contextvars.ContextVar("ftm_bound_comm", default=None)


def _cur() -> "Communicator | None":
    b = _BOUND.get()
    return b if b is not None else _COMM


@contextlib.contextmanager
def bound(c: "Communicator | None"):
    """Within the block (this thread), ``get()`` / ``is_dist()`` / the helpers below use
    ``c``: the communicator of the operator whose calls the block runs
    (``runtime/remote.py``: ``_GroupBound``)."""
    tok = _BOUND.set(c)
    try:
        yield c
    finally:
        _BOUND.reset(tok)


def init_distributed(communicator: type | None = None, timeout_s: int = 600, device=None) -> bool:
    """Creates the job's communicator when launched with WORLD_SIZE > 1 (RCCL on this
    rank's GPU).  ``communicator`` injects another implementation (tests: the loopback
    ``parallel.fake.FakeCommunicator``)."""
    global _COMM
    rank, ws, local = world()
    if _COMM is not None:
        return True
    if ws <= 1:
        return False
    store = rendezvous_store(rank, ws, timeout_s)
    if communicator is None:
        dev = torch.device("cuda", local_device(local)) if device is None else torch.device(device)
        _COMM = RcclCommunicator(rank, ws, dev, store)
    else:
        _COMM = communicator(rank, ws, device or "cpu", store)
    return True


def set_communicator(c: Communicator | None) -> None:
    """Installs ``c`` as the process's communicator (e.g. a world-size-1 RCCL communicator
    in GPU tests)."""
    global _COMM
    _COMM = c


def get() -> Communicator:
    c = _cur()
    if c is None:
        raise RuntimeError("no communicator: call init_distributed() under a launcher")
    return c


def destroy(abort: bool = False) -> None:
    """Tears down the communicator (``abort=True``: RCCL abort, no waiting on dead peers),
    so a restarted worker group can rendezvous afresh."""
    global _COMM
    if _COMM is not None:
        c, _COMM = _COMM, None
        c.destroy(abort=abort)


def is_dist() -> bool:
    """True when a communicator is installed (a world-size-1 RCCL communicator counts: its
    collectives still run through RCCL, e.g. in the GPU tests)."""
    return _cur() is not None


def rank_size() -> tuple[int, int]:
    c = _cur()
    return (c.rank, c.size) if c is not None else (0, 1)


def barrier():
    c = _cur()
    if c is not None:
        c.barrier()


def _bucket_plan(ts: Sequence[torch.Tensor], cap_elems: int):
    """Greedy packing of small tensors into buckets of at most ``cap_elems`` elements."""
    buckets, cur, n = [], [], 0
    for t in ts:
        if cur and n + t.numel() > cap_elems:
            buckets.append(cur)
            cur, n = [], 0
        cur.append(t)
        n += t.numel()
    if cur:
        buckets.append(cur)
    return buckets


def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0, comm: Communicator | None = None,
                      bucket_bytes: int = BROADCAST_BUCKET_BYTES) -> int:
    """In-place broadcast of many tensors from ``src``; returns the bytes broadcast.

    Tensors of at least a quarter bucket that are contiguous are broadcast where they live
    (zero extra memory); the rest are packed into one reusable staging bucket per dtype of
    ``bucket_bytes``.  Each round's calls are issued in one RCCL group."""
    c = comm or _cur()
    if c is None:
        return 0
    seen, by_dtype = set(), {}
    for t in tensors:  # plans of one arena share interned weights: send each storage once
        if t.numel() == 0 or t.data_ptr() in seen:
            continue
        seen.add(t.data_ptr())
        by_dtype.setdefault(t.dtype, []).append(t)
    total = 0
    for dt, ts in sorted(by_dtype.items(), key=lambda kv: str(kv[0])):
        esz = torch.empty((), dtype=dt).element_size()
        cap = max(1, bucket_bytes // esz)
        direct = [t for t in ts if t.is_contiguous() and t.numel() * 4 >= cap]
        small = [t for t in ts if not (t.is_contiguous() and t.numel() * 4 >= cap)]
        with c.group():
            for t in direct:
                c.broadcast(t, src)
        total += sum(t.numel() for t in direct) * esz
        if small:
            plan = _bucket_plan(small, cap)
            stage = torch.empty(min(cap, max(sum(t.numel() for t in b) for b in plan)), dtype=dt, device=c.device)
            for b in plan:
                n = sum(t.numel() for t in b)
                view = stage[:n]
                if c.rank == src:
                    torch.cat([t.reshape(-1) for t in b], out=view)
                c.broadcast(view, src)
                if c.rank != src:
                    off = 0
                    for t in b:
                        t.copy_(view[off:off + t.numel()].view_as(t))
                        off += t.numel()
                total += n * esz
    return total


def all_reduce_scalar(x: float, op: str = "sum", device=None) -> float:
    if not is_dist():
        return x
    c = _cur()
    t = torch.tensor([x], dtype=torch.float64, device=c.device)
    c.all_reduce(t, op)
    return float(t.item())


def all_gather_object(obj):
    if not is_dist():
        return [obj]
    return _cur().all_gather_object(obj)


def all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor) -> None:
    get().all_gather(out, inp)


class GradBucketer:
    """Bucketed, overlapped gradient all-reduce (DDP-style, written for xGMI rings).

    Parameters are assigned to buckets in reverse registration order (gradients become
    ready back-to-front).  When every gradient of a bucket has been produced, the bucket
    is flattened into its persistent flat buffer and an async RCCL all-reduce is launched
    on the communicator's stream while backward continues; ``synchronize()`` waits,
    averages and scatters the results back.  Sparse embedding gradients are handled by
    the embedding layer itself (row-sparse all-gather of touched rows) and are skipped."""

    def __init__(self, params: Sequence[torch.nn.Parameter], bucket_bytes: int = 25 << 20, average: bool = True,
                 comm: Communicator | None = None):
        self.params = [p for p in params if p.requires_grad]
        self.average = average
        # deferred: hooks only count; synchronize() launches every bucket in index order (an
        # agreed step where a rank without records has no backward, runtime/lockstep.py)
        self.deferred = False
        self.comm = comm or _cur()
        self.buckets: list[list[torch.nn.Parameter]] = []
        cur, cur_bytes = [], 0
        for p in reversed(self.params):
            nb = p.numel() * p.element_size()
            if cur and cur_bytes + nb > bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self._ready = [0] * len(self.buckets)
        self._handles: list = [None] * len(self.buckets)
        self._flat: list = [None] * len(self.buckets)
        self._hooks = []
        if self.comm is not None:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    @property
    def active(self) -> bool:
        return self.comm is not None

    def _on_grad(self, p):
        i = self._bucket_of[id(p)]
        self._ready[i] += 1
        if self._ready[i] == len(self.buckets[i]) and not self.deferred:
            self._launch(i)

    def _launch(self, i):
        b = self.buckets[i]
        flat = self._flat[i]
        if flat is None:
            flat = torch.empty(sum(p.numel() for p in b), dtype=b[0].dtype, device=b[0].device)
            self._flat[i] = flat
        off = 0
        for p in b:
            n = p.numel()
            if p.grad is None:
                flat[off:off + n].zero_()
            else:
                flat[off:off + n].copy_(p.grad.reshape(-1))
            off += n
        self._handles[i] = self.comm.all_reduce_async(flat, "sum")

    def synchronize(self):
        if not self.active:
            return
        ws = self.comm.size
        for i, b in enumerate(self.buckets):
            if self._handles[i] is None:  # some grads never produced (unused params)
                self._launch(i)
            self._handles[i].wait()
            flat = self._flat[i]
            if self.average:
                flat.div_(ws)
            off = 0
            for p in b:
                n = p.numel()
                g = flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
                off += n
            self._handles[i] = None
            self._ready[i] = 0

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()


def allgather_metrics(group) -> dict:
    """Whole-job metrics (SURVEY §2.13 ``allgather_metrics``): counters are summed and every
    latency histogram is merged bucket-wise across ranks, so p50/p99 are node-level
    percentiles.  Two collectives: the (small) name sets, then ONE int64 all-reduce holding
    all counters and all bucket vectors.  ``group`` is a ``utils.metrics.MetricGroup``.
    """
    from ..utils.metrics import BucketHistogram, histogram_buckets
    cnames = sorted(group.counters)
    hnames = sorted(group.histograms)
    if is_dist():
        names = all_gather_object((cnames, hnames))
        cnames = sorted({n for c, _ in names for n in c})
        hnames = sorted({n for _, h in names for n in h})
    vec = np.zeros(len(cnames) + len(hnames) * BucketHistogram.N, np.int64)
    for i, n in enumerate(cnames):
        vec[i] = group.counters.get(n, 0)
    for j, n in enumerate(hnames):
        if n in group.histograms:
            o = len(cnames) + j * BucketHistogram.N
            vec[o:o + BucketHistogram.N] = histogram_buckets(group.histograms[n]).counts
    if is_dist():
        c = _cur()
        t = torch.from_numpy(vec).to(c.device)
        c.all_reduce(t)
        vec = t.cpu().numpy()
    out = {"world_size": _cur().size if is_dist() else 1,
           "counters": {n: int(vec[i]) for i, n in enumerate(cnames)}, "histograms": {}}
    for j, n in enumerate(hnames):
        o = len(cnames) + j * BucketHistogram.N
        out["histograms"][n] = BucketHistogram(vec[o:o + BucketHistogram.N]).snapshot()
    return out
