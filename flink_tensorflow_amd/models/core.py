"""Model abstraction (SURVEY §2.2 M1–M4, §2.3 G1–G3).

* ``Model`` / ``RichModel`` — ``LIB/models/Model.scala:15-44``: a serializable descriptor;
  ``open()`` loads the graph and opens a session on the subtask's device before the first
  call, ``close()`` releases it.  Runtime fields are not pickled (the reference marks
  them ``@transient``), so models can be shipped to worker processes as descriptors.
* ``GraphMethod`` — ``LIB/graphs/GraphMethod.scala:8-36``: a typed method contract with a
  ``name`` that must equal the SignatureDef ``method_name``.
* ``ModelFunction`` — ``LIB/models/ModelFunction.scala:18-79``: binds (session, signature,
  method) into a callable.  Calling it returns a context manager over the outputs
  (``with model.fn(x) as y:``), the equivalent of the reference's lazy
  ``ManagedResource``; ``fn.apply(x)`` returns outputs directly.

  On a GPU session the signature is **compiled** (``graph/compiler.py``: MFMA conv/GEMM
  kernels, fused epilogues, hipGraph) once per feed-shape bucket and replayed: feeds are
  staged through pinned host buffers and copied H2D asynchronously into the plan's input
  buffers.  The leading (batch) dimension is padded up to the next of ``batch_buckets``
  (default 1, 2, 4, … 256), so a stream of varying micro-batch sizes reuses a handful of
  captured plans; outputs are sliced back.  Plans fold the session's variables into their
  weights and are recompiled when a variable is written (``VariableStore.version``).
  Signatures the compiler cannot take (STRING feeds such as serialized ``tf.Example``s,
  ops without a lowering and without a glue fallback) run on the op-by-op interpreter;
  ops lowered as PyTorch glue are logged and listed in ``plan_summary()["glue_ops"]``.
* ``GraphLoader`` / ``DefaultGraphLoader`` / ``GraphDefGraphLoader`` — ``LIB/graphs/*``.
* ``GenericModel`` — ``LIB/models/generic/GenericModel.scala:12-44``.
"""
from __future__ import annotations

import abc
import contextlib
import logging
from typing import Any, Callable, Mapping

import torch

from ..graph.graph import Graph
from ..graph.session import Session
from ..proto.messages import GraphDef, SignatureDef
from ..types.codecs import to_graph_tensor
from ..types.names import TensorName
from ..utils import fs

LOG = logging.getLogger("flink_tensorflow_amd.models")


class Model(abc.ABC):
    """Marker base for model descriptors (``Model[Self]``)."""

    _TRANSIENT: tuple[str, ...] = ()

    def __getstate__(self):
        st = dict(self.__dict__)
        for k in self._TRANSIENT:
            st[k] = None
        return st


class RichModel(Model):
    """A model with a lifecycle (``RichModel.open/close``)."""

    def open(self) -> None:  # noqa: B027 - optional hook
        pass

    def close(self) -> None:  # noqa: B027 - optional hook
        pass

    @property
    def is_open(self) -> bool:
        return True

    def __enter__(self):
        self.open()
        return self

    def __exit__(self, *a):
        self.close()


class CheckpointedModel(abc.ABC):
    """Model state that participates in checkpoints (repartitionable operator state) —
    ``LIB/streaming/models/CheckpointedModel.scala:24-46``.  ``ctx`` is the runtime's
    ``SnapshotContext`` / ``InitializationContext`` (``runtime/functions.py``)."""

    @abc.abstractmethod
    def snapshot_state(self, ctx) -> None:
        ...

    @abc.abstractmethod
    def initialize_state(self, ctx) -> None:
        ...


# ------------------------------------------------------------------ methods
class GraphMethod(abc.ABC):
    """Typed method: ``name`` + ``inputs(x) -> {signature key: tensor}`` +
    ``outputs({key: tensor}) -> result``."""

    name: str = ""

    @abc.abstractmethod
    def inputs(self, value) -> Mapping[str, Any]:
        ...

    @abc.abstractmethod
    def outputs(self, tensors: Mapping[str, Any]):
        ...


class BatchedGpuModel(abc.ABC):
    """Models that run micro-batches asynchronously on the GPU (pinned H2D on a side
    stream + hipGraph replay).  ``submit`` returns finished batches as
    ``(results, tags, latencies_s)``; ``drain`` waits for all in-flight batches."""

    @abc.abstractmethod
    def submit(self, records: list, ingest_ts: np.ndarray, tags: list) -> list:
        ...

    @abc.abstractmethod
    def poll(self) -> list:
        ...

    @abc.abstractmethod
    def drain(self) -> list:
        ...


class _Outputs(contextlib.AbstractContextManager):
    """Holds a call's outputs; closing releases them (arena slots / HBM references)."""

    def __init__(self, value):
        self.value = value
        self.closed = False

    def __enter__(self):
        return self.value

    def __exit__(self, *a):
        self.close()

    def close(self):
        self.value = None
        self.closed = True


DEFAULT_BATCH_BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256)


class ModelFunction:
    """``ModelFunction(session, signature_def, method)`` → callable.

    ``compile``: None = compile on GPU sessions, interpret on CPU; True/False force it.
    ``batch_buckets``: leading-dimension buckets of compiled plans (None: exact shapes).
    ``precision``: compiled-plan precision (``bf16`` or ``fp8``)."""

    def __init__(self, session_provider: Callable[[], Session] | Session, signature_def: SignatureDef,
                 method: GraphMethod, check_method_name: bool = True, compile: bool | None = None,
                 batch_buckets: tuple[int, ...] | None = DEFAULT_BATCH_BUCKETS, precision: str = "bf16",
                 strict: bool = False, pack_tokens: bool | None = None):
        if check_method_name and method.name and signature_def.method_name != method.name:
            raise ValueError(f"signature method name {signature_def.method_name!r} does not match "
                             f"method {method.name!r}")
        self._session = session_provider
        self.signature_def = signature_def
        self.method = method
        self._fetch_keys = sorted(signature_def.outputs)
        self._fetch_names = [str(TensorName.parse(signature_def.outputs[k].name)) for k in self._fetch_keys]
        self.compile = compile
        self.batch_buckets = tuple(sorted(batch_buckets)) if batch_buckets else None
        self.precision = precision
        self.strict = strict
        # token-id signatures whose attention masks come from the ids: padding-free plans
        # (graph/packed.py); None = whenever the graph allows it
        self.pack_tokens = pack_tokens
        self._plans: dict = {}          # feed-spec key -> (CompiledFunction, variables version, staging)
        self._interpret_reason: str | None = None
        self.last_plan = None

    @property
    def session(self) -> Session:
        s = self._session
        return s() if callable(s) and not isinstance(s, Session) else s

    def feeds(self, value, device=None) -> dict[str, Any]:
        sess = self.session
        mapped = self.method.inputs(value)
        feeds = {}
        for key, info in self.signature_def.inputs.items():
            if key not in mapped:
                raise ValueError(f"missing input {key!r} for signature (expected {sorted(self.signature_def.inputs)})")
            feeds[str(TensorName.parse(info.name))] = to_graph_tensor(
                mapped[key], device=sess.device if device is None else device)
        return feeds

    # ---------------------------------------------------------------- compiled path
    def _use_compiled(self, sess) -> bool:
        if self._interpret_reason is not None:
            return False
        return self.compile if self.compile is not None else sess.device.type == "cuda"

    def _bucket(self, feeds: dict) -> int | None:
        if not self.batch_buckets:
            return None
        lead = {int(v.shape[0]) for v in feeds.values() if isinstance(v, torch.Tensor) and v.dim() > 0}
        if len(lead) != 1 or any(not isinstance(v, torch.Tensor) or v.dim() == 0 for v in feeds.values()):
            return None
        n = lead.pop()
        return next((b for b in self.batch_buckets if b >= n), None)

    def _plan_for(self, sess, feeds: dict, bucket: int | None):
        from ..graph.compiler import compile_signature
        from ..types.dtypes import DataType

        specs = {k: ((bucket, *v.shape[1:]) if bucket else tuple(v.shape), DataType.from_torch(v.dtype))
                 for k, v in feeds.items()}
        key = tuple(sorted((k, sh, int(dt)) for k, (sh, dt) in specs.items()))
        version = getattr(sess.variables, "version", 0)
        hit = self._plans.get(key)
        if hit is not None and hit[1] == version:
            return hit
        plan = None
        if self.pack_tokens is not False and self.precision == "bf16" and bucket:
            from ..graph.packed import default_granule, try_packed

            (shape, _), = specs.values() if len(specs) == 1 else ((None, None),)
            if shape is not None and len(shape) == 2:
                plan = try_packed(sess.graph, specs, self._fetch_names, sess.device, variables=sess.variables,
                                  strict=self.strict, granule=default_granule(shape[0], shape[1]))
        if plan is None:
            plan = compile_signature(sess, specs, self._fetch_names, strict=self.strict, precision=self.precision)
        if plan.glue_ops:
            LOG.info("signature %s: ops run as PyTorch glue in the compiled plan: %s",
                     self.signature_def.method_name, sorted(set(plan.glue_ops)))
        pinned = sess.device.type == "cuda"
        staging = {k: torch.empty(sh, dtype=feeds[k].dtype, pin_memory=pinned).zero_() for k, (sh, _) in specs.items()}
        entry = (plan, version, staging)
        self._plans[key] = entry
        return entry

    def _run_compiled(self, sess, value):
        from ..graph.compiler import CompileError

        feeds = self.feeds(value, device=torch.device("cpu"))
        if any(not isinstance(v, torch.Tensor) for v in feeds.values()):
            self._interpret_reason = "non-tensor (STRING) feeds"
            LOG.info("signature %s runs on the interpreter: %s", self.signature_def.method_name,
                     self._interpret_reason)
            return None
        bucket = self._bucket(feeds)
        try:
            plan, _, staging = self._plan_for(sess, feeds, bucket)
        except (CompileError, NotImplementedError, KeyError, TypeError, ValueError) as e:
            self._interpret_reason = f"{type(e).__name__}: {e}"
            LOG.warning("signature %s cannot be compiled, using the interpreter: %s",
                        self.signature_def.method_name, self._interpret_reason)
            return None
        n = None
        for k, v in feeds.items():
            st = staging[k]
            if bucket:
                n = int(v.shape[0])
                st[:n].copy_(v)
                st[n:].zero_()  # no stale rows of an earlier, larger batch (packing counts tokens)
            else:
                st.copy_(v)
            if hasattr(plan, "select"):  # token-packed: capacity from the host-side ids
                plan.select(st, n)
            plan.input_buffer(k).copy_(st, non_blocking=True)
        outs = plan(None)
        if bucket:
            outs = [o[:n] if isinstance(o, torch.Tensor) and o.dim() > 0 and o.shape[0] == bucket else o for o in outs]
        self.last_plan = plan
        return outs

    def plan_summary(self) -> dict | None:
        """Summary of the most recently replayed compiled plan (None: interpreter)."""
        return self.last_plan.summary() if self.last_plan is not None else None

    @property
    def compiled_plans(self) -> int:
        return len(self._plans)

    # ---------------------------------------------------------------- call
    def run(self, value, run_metadata: bool = False):
        sess = self.session
        if self._use_compiled(sess):
            outs = self._run_compiled(sess, value)
            if outs is not None:
                out = self.method.outputs(dict(zip(self._fetch_keys, outs)))
                if run_metadata:
                    return out, self.last_plan.profile()
                return out
        res = sess.run(self._fetch_names, self.feeds(value), run_metadata=run_metadata)
        outs = res.outputs if run_metadata else res
        out = self.method.outputs(dict(zip(self._fetch_keys, outs)))
        if run_metadata:
            return out, res.metadata
        return out

    def apply(self, value):
        return self.run(value)

    def __call__(self, value) -> _Outputs:
        return _Outputs(self.run(value))


# ------------------------------------------------------------------ graph loaders
class GraphLoader(abc.ABC):
    @abc.abstractmethod
    def load(self) -> Graph:
        ...


class DefaultGraphLoader(GraphLoader):
    """Reads a binary GraphDef from a (URI) path, with an optional import prefix."""

    def __init__(self, path: str, prefix: str = ""):
        self.path = path
        self.prefix = prefix

    def load(self) -> Graph:
        data = fs.read_bytes(self.path)
        g = Graph.from_graph_def(data, self.prefix)
        LOG.info("loaded %s", self.path)
        return g


class GraphDefGraphLoader(GraphLoader):
    """Loads an in-memory GraphDef; the prefix IS applied (reference ignores it, B4)."""

    def __init__(self, graph_def: GraphDef | bytes, prefix: str = ""):
        self.graph_def_bytes = graph_def if isinstance(graph_def, bytes) else graph_def.encode()
        self.prefix = prefix

    def load(self) -> Graph:
        return Graph.from_graph_def(self.graph_def_bytes, self.prefix)


# ------------------------------------------------------------------ generic model
class GenericModel(RichModel):
    """A model over an ad-hoc graph.  Subclasses provide ``graph_loader``."""

    _TRANSIENT = ("_graph", "_session")

    def __init__(self, device: str | torch.device | None = None):
        self.device = device
        self._graph: Graph | None = None
        self._session: Session | None = None

    @property
    @abc.abstractmethod
    def graph_loader(self) -> GraphLoader:
        ...

    def open(self) -> None:
        if self._session is not None:
            return
        g = self.graph_loader.load()
        try:
            self._session = Session(g, device=self.device or default_device())
            self._graph = g
        except Exception:
            self._graph = None
            raise

    def close(self) -> None:
        if self._session is not None:
            self._session.close()
        self._session = None
        self._graph = None

    @property
    def is_open(self) -> bool:
        return self._session is not None

    def session(self) -> Session:
        if self._session is None:
            raise RuntimeError(f"{type(self).__name__} is not open")
        return self._session

    @property
    def graph(self) -> Graph:
        if self._graph is None:
            raise RuntimeError(f"{type(self).__name__} is not open")
        return self._graph


def default_device() -> torch.device:
    """The subtask's device: ``cuda:LOCAL_RANK`` when a GPU is visible, else CPU."""
    import os

    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", torch.cuda.current_device())))
    return torch.device("cpu")
