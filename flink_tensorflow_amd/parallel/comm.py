"""Collectives for data-parallel inference and online training.

One process per GPU; ``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm and
rides xGMI between the 8 MI355X of a node.  (``gloo`` is used only for CPU processes —
tests and host-only ranks.)  Collective call sites of the framework:

* ``broadcast_tensors``  — rank 0 loads / compiles the model, every other rank receives
  the weights in ONE flattened buffer per dtype (one RCCL broadcast instead of one per
  tensor; the root drives its 7 xGMI links in parallel);
* ``GradBucketer``       — bucketed gradient all-reduce for online training, launched
  from autograd hooks as buckets fill so communication overlaps backward (bucket size is
  chosen for per-link-bound rings on point-to-point xGMI, default 25 MB);
* ``barrier`` / ``all_gather_object`` / ``all_reduce_scalar`` — checkpoint alignment and
  metric aggregation (latency percentiles, records/s).
"""
from __future__ import annotations

import datetime
import os
from typing import Iterable, Sequence

import numpy as np
import torch
import torch.distributed as dist


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
    import os

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


def init_distributed(backend: str | None = None, timeout_s: int = 600) -> bool:
    """Initialises the default process group when launched with WORLD_SIZE > 1."""
    rank, ws, local = world()
    if ws <= 1 or dist.is_initialized():
        return dist.is_initialized()
    if backend is None:
        # FTM_DIST_BACKEND=gloo rehearses the multi-rank flow with several ranks sharing
        # one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("FTM_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local_device(local))
        kw["device_id"] = torch.device("cuda", local_device(local))
    dist.init_process_group(backend, rank=rank, world_size=ws, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return True


def destroy() -> None:
    """Tears down the process group (RCCL communicator abort + free on the GPU path), so
    a restarted worker group can rendezvous afresh."""
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def barrier():
    if is_dist():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def _flatten(ts: Sequence[torch.Tensor]) -> torch.Tensor:
    return torch.cat([t.reshape(-1) for t in ts]) if ts else torch.empty(0)


def _unflatten_into(flat: torch.Tensor, ts: Sequence[torch.Tensor]):
    off = 0
    for t in ts:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t))
        off += n


def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0) -> int:
    """In-place broadcast of many tensors from ``src``: one flattened buffer per dtype.
    Returns the number of bytes broadcast."""
    if not is_dist():
        return 0
    by_dtype: dict = {}
    seen = set()
    for t in tensors:  # plans of one arena share interned weights: send each storage once
        if t.data_ptr() in seen and t.numel():
            continue
        seen.add(t.data_ptr())
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    total = 0
    for (dt, dev), ts in sorted(by_dtype.items(), key=lambda kv: str(kv[0])):
        flat = _flatten(ts).contiguous()
        dist.broadcast(flat, src)
        if dist.get_rank() != src:
            _unflatten_into(flat, ts)
        total += flat.numel() * flat.element_size()
    return total


def all_reduce_scalar(x: float, op: str = "sum", device=None) -> float:
    if not is_dist():
        return x
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op])
    return float(t.item())


def all_gather_object(obj):
    if not is_dist():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


class GradBucketer:
    """Bucketed, overlapped gradient all-reduce (DDP-style, written for xGMI rings).

    Parameters are assigned to buckets in reverse registration order (gradients become
    ready back-to-front).  When every gradient of a bucket has been produced, the bucket
    is flattened and an async all-reduce is launched on the process group while backward
    continues; ``synchronize()`` waits, averages and scatters the results back.
    Sparse embedding gradients are handled by the embedding layer itself (row-sparse
    all-reduce of touched rows) and are skipped here.
    """

    def __init__(self, params: Sequence[torch.nn.Parameter], bucket_bytes: int = 25 << 20, average: bool = True):
        self.params = [p for p in params if p.requires_grad]
        self.average = average
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
        if is_dist():
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    def _on_grad(self, p):
        i = self._bucket_of[id(p)]
        self._ready[i] += 1
        if self._ready[i] == len(self.buckets[i]):
            self._launch(i)

    def _launch(self, i):
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in self.buckets[i]]
        flat = _flatten(grads).contiguous()
        self._flat[i] = flat
        self._handles[i] = dist.all_reduce(flat, async_op=True)

    def synchronize(self):
        if not is_dist():
            return
        ws = dist.get_world_size()
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
            self._flat[i] = None
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
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
        t = torch.from_numpy(vec).to(dev)
        dist.all_reduce(t)
        vec = t.cpu().numpy()
    out = {"world_size": dist.get_world_size() if is_dist() else 1,
           "counters": {n: int(vec[i]) for i, n in enumerate(cnames)}, "histograms": {}}
    for j, n in enumerate(hnames):
        o = len(cnames) + j * BucketHistogram.N
        out["histograms"][n] = BucketHistogram(vec[o:o + BucketHistogram.N]).snapshot()
    return out
