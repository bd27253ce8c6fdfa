"""Per-subtask tensor arena (SURVEY §2.8 N1, §5.6 ``arena fraction of 288 GB``).

The reference moves every record through fresh native buffers per ``Session.run``
(``LIB/types/TensorValue.java:131-133,257-263``; four JNI copies per image).
Here a GPU subtask owns ONE ``DeviceArena`` whose budget is its share of the MI355X's
288 GB of HBM (``EngineConfig.arena_bytes``); everything the subtask's compiled plans and
staging ring touch is carved out of it:

* **activation slab** — a compiled plan's intermediate tensors get byte offsets in one slab
  from the native liveness planner (``_native.plan_offsets``: tensors alive at the same
  step never overlap).  Plans of one subtask run serially on its compute stream, so all
  their batch buckets SHARE the slab (``shared_slab``): the 64/128/256-row ResNet plans
  cost max(slab) instead of sum(slab) of HBM;
* **persistent blocks** — feed/fetch buffers and weights, sub-allocated by the native
  first-fit ``OffsetAllocator`` (coalescing free list) from large chunks;
* **interned weights** — identical device weights of several bucket plans (the same folded
  BN conv filter compiled 4x for 4 buckets) are stored once (``intern``).

Every byte is charged against the budget; exceeding it raises ``ArenaExhausted`` at
compile time instead of an allocator failure mid-stream.  ``stats()`` reports usage (the
per-GPU HBM arena metric of SURVEY §5.5).
"""
from __future__ import annotations

import hashlib
import threading

import numpy as np
import torch

from .. import _ext

_ALIGN = 256  # bytes; >= the 16-B alignment every HIP kernel checks, and a full L2 line pair
_CHUNK = 256 << 20


class ArenaExhausted(MemoryError):
    pass


def _nbytes(shape, dtype) -> int:
    return int(np.prod(shape, dtype=np.int64)) * torch.empty((), dtype=dtype).element_size()


class DeviceArena:
    """HBM arena of one subtask (``device`` may be ``cpu`` for host plans in tests)."""

    def __init__(self, device, budget_bytes: int | None = None, chunk_bytes: int = _CHUNK, name: str = ""):
        self.device = torch.device(device)
        if budget_bytes is None:
            from ..config import EngineConfig

            budget_bytes = EngineConfig().arena_bytes(self.device if self.device.type == "cuda" else None)
        self.budget = int(budget_bytes)
        self.chunk_bytes = int(chunk_bytes)
        self.name = name
        self._lock = threading.Lock()
        self._chunks: list[tuple[torch.Tensor, object]] = []  # (uint8 storage, OffsetAllocator)
        self._owner: dict[int, tuple[int, int]] = {}  # data_ptr -> (chunk index, offset)
        self._slab: torch.Tensor | None = None
        self._retired_slab_bytes = 0  # slabs replaced by a larger one, still referenced by older plans
        self._interned: dict[tuple, torch.Tensor] = {}
        self.interned_hits = 0

    # ------------------------------------------------------------------ accounting
    @property
    def reserved(self) -> int:
        chunks = sum(c.numel() for c, _ in self._chunks)
        slab = self._slab.numel() if self._slab is not None else 0
        return chunks + slab + self._retired_slab_bytes

    def _charge(self, nbytes: int, what: str):
        if self.reserved + nbytes > self.budget:
            raise ArenaExhausted(f"arena {self.name or self.device}: {what} needs {nbytes / 2**20:.1f} MiB; "
                                 f"{self.reserved / 2**20:.1f} of {self.budget / 2**20:.1f} MiB reserved")

    # ------------------------------------------------------------------ activation slab
    def shared_slab(self, nbytes: int) -> torch.Tensor:
        """A uint8 region of at least ``nbytes`` shared by every plan of this subtask.
        Growing it allocates a new slab; plans bound to the old one keep it alive."""
        with self._lock:
            if self._slab is None or self._slab.numel() < nbytes:
                old = self._slab.numel() if self._slab is not None else 0
                self._charge(nbytes - old, "activation slab")
                if self._slab is not None:
                    self._retired_slab_bytes += old
                self._slab = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=self.device)
            return self._slab

    # ------------------------------------------------------------------ persistent blocks
    def alloc(self, shape, dtype) -> torch.Tensor:
        nb = max(_nbytes(shape, dtype), 1)
        native = _ext.native()
        with self._lock:
            for ci, (buf, al) in enumerate(self._chunks):
                off = al.alloc(nb)
                if off >= 0:
                    break
            else:
                size = max(self.chunk_bytes, -(-nb // _ALIGN) * _ALIGN)
                self._charge(size, "persistent chunk")
                buf = torch.empty(size, dtype=torch.uint8, device=self.device)
                al = native.OffsetAllocator(size, _ALIGN)
                self._chunks.append((buf, al))
                ci, off = len(self._chunks) - 1, al.alloc(nb)
            t = buf[off:off + nb].view(dtype).view(tuple(shape))
            self._owner[t.data_ptr()] = (ci, off)
            return t

    def free(self, t: torch.Tensor) -> None:
        with self._lock:
            ci, off = self._owner.pop(t.data_ptr())
            self._chunks[ci][1].free(off)

    def intern(self, t: torch.Tensor) -> torch.Tensor:
        """Device copy of ``t`` (host or device), shared with earlier identical tensors."""
        host = t.detach().to("cpu").contiguous()
        raw = host.view(-1).view(torch.uint8).numpy() if host.numel() else b""
        key = (tuple(host.shape), host.dtype, hashlib.blake2b(raw, digest_size=16).hexdigest())
        with self._lock:
            hit = self._interned.get(key)
        if hit is not None:
            self.interned_hits += 1
            return hit
        dev = self.alloc(host.shape, host.dtype)
        dev.copy_(host)
        with self._lock:
            self._interned[key] = dev
        return dev

    def stats(self) -> dict:
        with self._lock:
            return {"budget_bytes": self.budget, "reserved_bytes": self.reserved,
                    "slab_bytes": self._slab.numel() if self._slab is not None else 0,
                    "retired_slab_bytes": self._retired_slab_bytes,
                    "persistent_in_use_bytes": sum(al.in_use for _, al in self._chunks),
                    "persistent_chunks": len(self._chunks), "interned_tensors": len(self._interned),
                    "interned_hits": self.interned_hits}


def plan_offsets(sizes, first, last, align: int = _ALIGN) -> tuple[list[int], int]:
    """Native liveness offset planner (see ``csrc/arena.cpp``)."""
    offs, total = _ext.native().plan_offsets([int(s) for s in sizes], [int(f) for f in first],
                                              [int(v) for v in last], align)
    return list(offs), int(total)
