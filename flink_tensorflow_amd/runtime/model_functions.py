"""Model-aware stream functions (SURVEY §2.5 F1–F10).

* ``ModelAwareFunction`` — ``LIB/common/functions/util/ModelAwareFunction.scala``: opens
  the model in ``open`` (binding the subtask's GPU first) and closes it in ``close``.
  Models that are not ``RichModel``s are simply used (the reference's non-exhaustive match
  throws ``MatchError``, B6).
* ``CheckpointedModel`` — ``LIB/streaming/models/CheckpointedModel.scala:24-46``;
  ``CheckpointedModelAwareFunction`` connects it to the checkpoint barriers with a
  **no-op default** for stateless models (B6).  ``TensorFlowModel``
  (``models/savedmodel.py``: session variables) and the online-training
  ``WideDeepTrainer`` (``models/zoo/wide_deep.py``: weights + optimizer state) implement
  it; both write TensorBundle V2 under ``chk-N/models/``.
* ``Model{Map,FlatMap,Process,CoProcess,Window,AllWindow}Function`` —
  ``Abstract*Function`` of ``LIB/common/functions`` and ``LIB/streaming/functions``.
* ``BatchedModelOperator`` — the micro-batching operator behind
  ``DataStream.map_with_model_batched`` (no reference analogue: the reference runs
  batch 1 per record, B9).
"""
from __future__ import annotations

import os
import time

import numpy as np

from ..models.core import BatchedGpuModel, CheckpointedModel, RichModel  # noqa: F401  (re-exported)
from . import functions as F
from .operators import Operator, Record




def open_model(model, device=None):
    """``ModelUtils.openModel`` with exhaustive dispatch."""
    if isinstance(model, RichModel):
        if device is not None and getattr(model, "device", None) is None and hasattr(model, "device"):
            model.device = device
        if not model.is_open:
            model.open()


def close_model(model):
    if isinstance(model, RichModel) and model.is_open:
        model.close()


class ModelAwareFunction(F.RichFunction):
    """Mixin: a function that owns a model descriptor (``self.model``)."""

    def __init__(self, model=None):
        F.RichFunction.__init__(self)
        if model is not None:
            self.model = model

    def open(self, config=None):
        ctx = getattr(self, "_runtime_context", None)
        if ctx is not None and hasattr(self.model, "restart_attempt"):
            self.model.restart_attempt = ctx.attempt  # models that adapt after a failure
            self.model.restart_budget = getattr(ctx, "restart_attempts", None)
        open_model(self.model, ctx.device if ctx is not None else None)

    def close(self):
        close_model(self.model)


class CheckpointedModelAwareFunction(ModelAwareFunction, F.CheckpointedFunction):
    """Forwards ``snapshot_state``/``initialize_state`` to a ``CheckpointedModel``; no-op
    for other models (instead of ``MatchError``)."""

    def snapshot_state(self, ctx):
        if isinstance(self.model, CheckpointedModel):
            self.model.snapshot_state(ctx)

    def initialize_state(self, ctx):
        if isinstance(self.model, CheckpointedModel):
            self.model.initialize_state(ctx)


class ModelMapFunction(ModelAwareFunction, F.MapFunction):
    """``AbstractMapFunction`` (no checkpointing)."""


class ModelFlatMapFunction(ModelAwareFunction, F.FlatMapFunction):
    """``AbstractFlatMapFunction``."""


class ModelProcessFunction(CheckpointedModelAwareFunction, F.ProcessFunction):
    """``AbstractProcessFunction``."""


class ModelCoProcessFunction(CheckpointedModelAwareFunction, F.CoProcessFunction):
    """``AbstractCoProcessFunction`` — the home of online training (data + update streams)."""


class ModelWindowFunction(CheckpointedModelAwareFunction, F.WindowFunction):
    """``AbstractWindowFunction`` — a window is a natural micro-batch."""


class ModelAllWindowFunction(CheckpointedModelAwareFunction, F.AllWindowFunction):
    """``AbstractAllWindowFunction``."""


# ------------------------------------------------------------------ micro-batching
class BatchedModelOperator(Operator):
    def __init__(self, model, batch_fn, max_batch: int, max_delay_ms: float, name: str, emit_batches: bool = False):
        super().__init__(None, name)
        from ..batching.engine import MicroBatcher

        self.model = model
        self.batch_fn = batch_fn
        self.batcher = MicroBatcher(max_batch, max_delay_ms)
        self.emit_batches = emit_batches
        self._ts_of: list = []

    def open(self):
        open_model(self.model, self.ctx.device)
        if isinstance(self.model, F.RichFunction):
            self.model.set_runtime_context(self.ctx)

    def close(self):
        close_model(self.model)

    def initialize(self, snapshot, checkpoint_dir):
        super().initialize(snapshot, checkpoint_dir)
        if isinstance(self.model, CheckpointedModel):
            self.model.initialize_state(F.InitializationContext(self.op_state, snapshot is not None, checkpoint_dir,
                                                                self.ctx.subtask_index))

    def process(self, rec: Record, input_index=0):
        b = self.batcher.add(rec, time.perf_counter())
        if b is not None:
            self._run(*b)

    def process_many(self, values: list, ts=None):
        """A run of records from a chained bulk source (``SourceContext.collect_many``)."""
        for b in self.batcher.add_many([Record(v, ts) for v in values], time.perf_counter()):
            self._run(*b)

    def _run(self, recs, ts):
        m = self.ctx.metrics
        if m is not None:
            m.histogram("batch_size").update(len(recs))
        if isinstance(self.model, BatchedGpuModel) and self.batch_fn is None:
            done = self.model.submit([r.value for r in recs], ts, [r.ts for r in recs])
            self._emit_done(done)
        else:
            out = self.batch_fn(self.model, [r.value for r in recs])
            lat = time.perf_counter() - ts
            if m is not None:
                m.histogram("latency_s").update_many(lat)
            if self.emit_batches:
                self.out.emit(out, recs[-1].ts)
            else:
                if len(out) != len(recs):
                    raise ValueError(f"batch function returned {len(out)} results for {len(recs)} records")
                for r, o in zip(recs, out):
                    self.out.emit(o, r.ts)

    def _emit_done(self, done):
        m = self.ctx.metrics
        for results, tags, lat in done:
            if m is not None:
                m.histogram("latency_s").update_many(lat)
            if self.emit_batches:
                self.out.emit(results, tags[-1] if tags else None)
            else:
                for o, t in zip(results, tags):
                    self.out.emit(o, t)

    def on_idle(self, now):
        if self.batcher.due():
            b = self.batcher.flush()
            if b is not None:
                self._run(*b)
        if isinstance(self.model, BatchedGpuModel):
            self._emit_done(self.model.poll())

    def next_deadline(self):
        if not self.batcher.items:
            return None
        return time.time() + max(0.0, self.batcher.max_delay - (time.perf_counter() - self.batcher.ts[0]))

    def _flush_all(self):
        b = self.batcher.flush()
        if b is not None:
            self._run(*b)
        if isinstance(self.model, BatchedGpuModel):
            self._emit_done(self.model.drain())

    def prepare_snapshot(self):
        self._flush_all()  # a batch never straddles a barrier

    def snapshot_state(self, checkpoint_id, checkpoint_dir):
        if isinstance(self.model, CheckpointedModel):
            self.model.snapshot_state(F.SnapshotContext(checkpoint_id, time.time(), self.op_state, checkpoint_dir,
                                                        self.ctx.subtask_index))
        return super().snapshot_state(checkpoint_id, checkpoint_dir)

    def end_input(self):
        self._flush_all()


class InputFormatModelOperations:
    """Source-side model lifecycle (``LIB/common/io/InputFormatModelOperations.scala``):
    mix into a ``WholeFileInputFormat`` that owns ``self.model``."""

    def open_input_format(self):
        open_model(self.model)

    def close_input_format(self):
        close_model(self.model)


def model_state_dir(ctx, name: str) -> str | None:
    """Per-subtask directory inside a checkpoint for model bundles."""
    if ctx.checkpoint_dir is None:
        return None
    d = os.path.join(ctx.checkpoint_dir, "models", f"{name}-{ctx.subtask_index}")
    os.makedirs(d, exist_ok=True)
    return d
