"""Padding-free execution of a compiled transformer signature (BERT-style SavedModels).

``PackedFunction`` compiles one ``CompiledFunction(token_capacity=T)`` per token capacity T
(multiples of ``granule`` up to batch*seq) of the same (graph, feeds, fetches) signature,
all on one ``DeviceArena`` (one shared activation slab, weights interned once).  Per
micro-batch, ``select(host_ids, n)`` counts the real tokens on the HOST — from the pinned
staging slot the runner already holds, so no device synchronisation — and picks the
smallest capacity that holds them; the plan's own ``pack_tokens`` kernel then compacts the
same tokens on the device.  Every projection, LayerNorm and attention runs on the packed
rows only, and the final layer after its QKV projection on one row per sequence
(``graph/transformer_lowering.py``).

It implements the plan protocol of ``batching.engine.PipelinedGpuRunner``
(``input_buffer`` / ``replay`` / ``output_tensors`` / ``select``) and ``__call__`` like a
``CompiledFunction``.  The reference runs the same signature per record through
``ModelFunction`` (``ModelFunction.scala:34-79``), where every padding token costs a full
row of every matmul.
"""
from __future__ import annotations

import numpy as np
import torch

from ..types.names import TensorName
from .compiler import CompiledFunction, CompileError


class PackedFunction:
    def __init__(self, graph, feeds: dict, fetches: list[str], device, variables: dict | None = None,
                 use_graph: bool = True, strict: bool = False, arena=None, granule: int = 2048,
                 capacities=None):
        if len(feeds) != 1:
            raise CompileError("token packing takes exactly one feed (the token ids)")
        (feed, (shape, _)), = feeds.items()
        if len(shape) != 2:
            raise CompileError("token packing needs [batch, seq] ids")
        self.feed = str(TensorName.parse(feed))
        self.B, self.S = int(shape[0]), int(shape[1])
        full = self.B * self.S
        if capacities is None:
            g = max(16, min(int(granule), full))
            capacities = range(g, full + g, g)
        self.caps = sorted({min(full, int(c)) for c in capacities} | {full})
        self.plans: dict[int, CompiledFunction] = {}
        for c in reversed(self.caps):  # largest first: every capacity shares the first slab
            self.plans[c] = CompiledFunction(graph, feeds, fetches, device, variables, use_graph=use_graph,
                                             strict=strict, arena=arena, token_capacity=c)
        self.plans = dict(sorted(self.plans.items()))
        self.pad = self.plans[full]._pack["pad"]
        self.current = self.plans[full]
        self.params = list({t.data_ptr(): t for p in self.plans.values() for t in p.params}.values())

    # ---------------------------------------------------------------- selection
    def capacity_for(self, n_tokens: int) -> int:
        for c in self.caps:
            if c >= n_tokens:
                return c
        raise ValueError(f"{n_tokens} tokens exceed batch*seq = {self.caps[-1]}")

    def select(self, host_ids, n: int | None = None) -> CompiledFunction:
        a = host_ids.numpy() if isinstance(host_ids, torch.Tensor) else np.asarray(host_ids)
        self.current = self.plans[self.capacity_for(int(np.count_nonzero(a != self.pad)))]
        return self.current

    # ---------------------------------------------------------------- plan protocol
    def input_buffer(self, feed: str) -> torch.Tensor:
        return self.current.input_buffer(feed)

    def replay(self):
        self.current.replay()

    def output_tensors(self) -> list:
        return self.current.output_tensors()

    def __call__(self, feeds: dict | None = None, copy_outputs: bool = True, cast_outputs: bool = True):
        """With ``feeds`` the capacity is selected from the ids (one host copy); without,
        the current plan runs on what ``input_buffer`` holds (``select`` called before)."""
        if feeds:
            ids = feeds.get(self.feed, next(iter(feeds.values())))
            self.select(ids.detach().cpu() if isinstance(ids, torch.Tensor) else ids)
        return self.current(feeds, copy_outputs, cast_outputs)

    @property
    def glue_ops(self) -> list:
        return sorted({g for p in self.plans.values() for g in p.glue_ops})

    def profile(self, feeds: dict | None = None):
        return self.current.profile(feeds)

    def summary(self) -> dict:
        s = dict(self.plans[self.caps[-1]].summary())
        s["token_capacities"] = list(self.caps)
        s["packed"] = True
        return s

    def param_bytes(self) -> int:
        return sum(p.numel() * p.element_size() for p in self.params)


def packable_feeds(feeds: dict) -> bool:
    """One rank-2 integer feed ([batch, seq] token ids): the signatures token packing serves."""
    if len(feeds) != 1:
        return False
    (shape, dt), = feeds.values()
    from ..types.dtypes import DataType

    return len(shape) == 2 and DataType.of(dt).torch in (torch.int32, torch.int64) and int(shape[1]) > 1


def default_granule(batch: int, seq: int) -> int:
    """Token-capacity step: 2048 tokens, but at most 16 capacities per batch bucket (BERT-base
    at B=256 x 128: 16 plans; the 4096 step of 8 plans pads ~8 % more tokens and measured 7 %
    slower end to end, profiles/r06_jobs)."""
    return max(2048, -(-batch * seq // 16))


def try_packed(graph, feeds: dict, fetches: list[str], device, **kw) -> PackedFunction | None:
    """A ``PackedFunction`` when the signature can run token-packed, else None (the caller
    keeps its padded plan)."""
    if not packable_feeds(feeds):
        return None
    try:
        return PackedFunction(graph, feeds, fetches, device, **kw)
    except CompileError:
        return None
