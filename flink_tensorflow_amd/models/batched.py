"""A SavedModel signature as a pipelined micro-batch model.

``ModelFunction`` (``models/core.py``) runs one call at a time: stage, replay, wait.  For a
stream of single records that is the reference's ``ModelFunction.run`` per record
(``flink-tensorflow/.../models/ModelFunction.scala:44-66``) batched, but still serial on the
GPU.  ``SignatureBatchedModel`` serves the same signature of ANY user SavedModel through the
runner the zoo models use (``batching/engine.py::PipelinedGpuRunner``): per batch bucket and
per compute lane one compiled plan (hand-written kernels, hipGraph, one ``DeviceArena``
per lane), host gather into pinned slots, H2D on a copy stream, lanes replaying
concurrently, results harvested in submission order.  ``DataStream.map_with_model_batched``
picks that path for any ``BatchedGpuModel`` when no batch function is given.

Limits (checked at open): one input tensor per record, with a static per-record shape
(from the signature, or ``record_shape``); outputs batched on the leading dimension.
Variables assigned after compile (``sess.variables.version``) trigger a drain and a
recompile, like ``ModelFunction``.  On a host device records run on the interpreter.
"""
from __future__ import annotations

import logging
import time
from typing import Sequence

import numpy as np
import torch

from ..types.dtypes import DataType
from ..types.names import TensorName
from ..types.tensor_value import TensorValue
from .core import BatchedGpuModel
from .savedmodel import TAG_SERVE, SavedModel_, SignatureConstants

LOG = logging.getLogger(__name__)


class SignatureBatchedModel(SavedModel_, BatchedGpuModel):
    """``SignatureBatchedModel(path, signature, buckets=(64, 256), lanes=2)``: records are
    single input tensors; each result is ``{output_key: row}`` (numpy)."""

    _TRANSIENT = SavedModel_._TRANSIENT + ("_plans", "_runner", "_arena", "_version")

    def __init__(self, path: str, signature: str = SignatureConstants.DEFAULT_SERVING_SIGNATURE_DEF_KEY,
                 input_key: str | None = None, output_keys: Sequence[str] | None = None,
                 record_shape: Sequence[int] | None = None, buckets: Sequence[int] = (64, 256), lanes: int = 2,
                 depth: int = 3, precision: str = "bf16", tags: Sequence[str] = (TAG_SERVE,), device=None,
                 distributed_weights: bool = False, pack_tokens: bool | None = None, lane_offset_us: float = 0.0):
        super().__init__(path, tags, device, distributed_weights)
        # staggered start of the compute lanes (batching/engine.py ``lane_offset_us``)
        self.lane_offset_us = float(lane_offset_us)
        # token-id signatures (BERT-style, mask computed from the ids): padding-free plans
        # (graph/packed.py).  None = whenever the graph allows it, False = padded plans
        self.pack_tokens = pack_tokens
        self.signature = signature
        self.input_key = input_key
        self.output_keys = list(output_keys) if output_keys is not None else None
        self.record_shape = tuple(record_shape) if record_shape is not None else None
        self.buckets = tuple(sorted(int(b) for b in buckets))
        self.lanes = max(1, int(lanes))
        self.depth = depth
        self.precision = precision
        self._plans = None
        self._runner = None
        self._arena = None
        self._version = None

    # ------------------------------------------------------------------ signature
    def _io(self):
        sd = self.signature_def(self.signature)
        if sd is None:
            raise KeyError(f"no signature {self.signature!r}; available: {sorted(self.metagraph.signature_def)}")
        keys = list(sd.inputs)
        key = self.input_key or (keys[0] if len(keys) == 1 else None)
        if key is None or key not in sd.inputs:
            raise ValueError(f"signature {self.signature!r} has inputs {keys}: pass input_key= (one input per record)")
        info = sd.inputs[key]
        shape = self.record_shape
        if shape is None:
            ts = info.tensor_shape
            dims = [int(d.size) for d in ts.dim] if ts is not None and not ts.unknown_rank else None
            if not dims or any(d < 0 for d in dims[1:]):
                raise ValueError(f"input {key!r} has no static per-record shape ({dims}): pass record_shape=")
            shape = tuple(dims[1:])
        outs = self.output_keys or sorted(sd.outputs)
        return (str(TensorName.parse(info.name)), DataType(int(info.dtype)), shape, outs,
                [str(TensorName.parse(sd.outputs[k].name)) for k in outs])

    # ------------------------------------------------------------------ lifecycle
    def open(self) -> None:
        super().open()
        self._feed, self._dtype, self._shape, self._out_keys, self._fetches = self._io()
        if self.session().device.type == "cuda":
            self._compile()

    def _compile(self) -> None:
        from ..batching.arena import DeviceArena
        from ..batching.engine import PipelinedGpuRunner
        from ..config import EngineConfig
        from ..graph.compiler import CompiledFunction
        from ..graph.packed import default_granule, try_packed

        sess = self.session()
        dev = sess.device
        budget = EngineConfig().arena_bytes(dev) // self.lanes
        self._arena = [DeviceArena(dev, budget, name=f"{self.signature}/lane{i}") for i in range(self.lanes)]

        def plan(b, arena):
            spec = {self._feed: ((b, *self._shape), self._dtype.name)}
            if self.pack_tokens is not False and self.precision == "bf16":
                p = try_packed(sess.graph, spec, self._fetches, dev, variables=sess.variables, arena=arena,
                               granule=default_granule(b, self._shape[0]) if self._shape else 2048)
                if p is not None:
                    return p
                if self.pack_tokens:
                    raise ValueError(f"signature {self.signature!r} cannot run token-packed")
            return CompiledFunction(sess.graph, spec, self._fetches, dev, sess.variables, strict=False,
                                    precision=self.precision, arena=arena)

        lanes = [{b: plan(b, arena) for b in sorted(self.buckets, reverse=True)} for arena in self._arena]
        self._plans = lanes[0]
        glue = sorted({g for p in self._plans.values() for g in p.glue_ops})
        if glue:
            LOG.info("signature %s: ops run as PyTorch glue in the compiled plans: %s", self.signature, glue)
        self._runner = PipelinedGpuRunner(lanes, self._feed, lambda p: p.output_tensors(), self._shape,
                                          self._dtype.torch, depth=self.depth, device=dev,
                                          lane_offset_us=getattr(self, "lane_offset_us", 0.0))
        self._version = getattr(sess.variables, "version", 0)

    def close(self) -> None:
        if self._runner is not None:
            self._runner.drain()
        self._runner = self._plans = self._arena = None
        super().close()

    def plan_summary(self) -> dict | None:
        return next(iter(self._plans.values())).summary() if self._plans else None

    # ------------------------------------------------------------------ batched GPU API
    def _as_array(self, r) -> np.ndarray:
        if isinstance(r, TensorValue):
            r = r.to_numpy()
        elif isinstance(r, torch.Tensor):
            r = r.cpu().numpy()
        a = np.ascontiguousarray(r, dtype=self._dtype.numpy)
        if a.shape != self._shape:
            a = a.reshape(self._shape)  # raises on a record of the wrong size
        return a

    def _rows(self, outs, n):
        cols = [o[:n].float().numpy() if o.dtype == torch.bfloat16 else o[:n].numpy() for o in outs]
        return [{k: c[i] for k, c in zip(self._out_keys, cols)} for i in range(n)]

    def _results(self, br):
        return self._rows(br.outputs, br.n), br.tags, br.latencies

    def submit(self, records, ingest_ts, tags):
        arrs = [self._as_array(r) for r in records]
        if self._runner is None:  # host: synchronous interpreter run
            outs = self.session().run(self._fetches, {self._feed: torch.from_numpy(np.stack(arrs))})
            return [(self._rows([o.cpu() for o in outs], len(arrs)), list(tags),
                     time.perf_counter() - np.asarray(ingest_ts))]
        done = []
        if getattr(self.session().variables, "version", 0) != self._version:  # weights assigned since compile
            done = [self._results(b) for b in self._runner.drain()]
            self._compile()
        cap = self.buckets[-1]
        for s in range(0, len(arrs), cap):
            for br in self._runner.submit(arrs[s:s + cap], np.asarray(ingest_ts[s:s + cap]), list(tags[s:s + cap])):
                done.append(self._results(br))
        return done

    def poll(self):
        return [self._results(b) for b in self._runner.poll()] if self._runner is not None else []

    def drain(self):
        return [self._results(b) for b in self._runner.drain()] if self._runner is not None else []
