"""``Session``: feeds → fetches/targets execution over a :class:`Graph`.

Replaces libtensorflow's ``TF_NewSession``/``TF_SessionRun`` as driven by the reference
(``LIB/models/generic/GenericModel.scala:25``, ``LIB/models/ModelFunction.scala:47-65``,
``LIB/io/Saver.scala:62-65,82-85``).  Semantics kept: pruning to the fetched/targeted
subgraph, feeding any tensor by ``"op:idx"`` name, control dependencies (``^name``),
variables with Assign, and an optional per-node step trace (``run_and_fetch_metadata``:
the reference calls ``runAndFetchMetadata`` but never sets a trace level).

Plans (pruned + topologically ordered node lists) are cached per (feeds, fetches,
targets) signature, so the per-record cost is a dictionary walk, not graph analysis.
For the hot GPU path, ``compile_signature`` (``compiler.py``) lowers a plan onto the
hand-written kernels and captures it in a hipGraph.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Any, Mapping, Sequence

import torch

from ..proto.messages import DeviceStepStats, NodeExecStats, RunMetadata, StepStats
from ..types.names import TensorName
from ..types.tensor import StringTensor, as_tensor
from . import control_flow, ops_core, ops_io, ops_nn  # noqa: F401  (register kernels)
from .graph import Graph
from .op_registry import REF_INPUT_OPS, OpContext, lookup


@dataclass
class _Plan:
    order: list[str]
    fed_nodes: frozenset
    control_flow: bool = False  # Switch/Merge/Enter/...: tagged-token dataflow (control_flow.py)
    topology: Any = None


class Run:
    """Result of ``Runner.run_and_fetch_metadata`` (TF Java ``Session.Run``)."""

    def __init__(self, outputs, metadata: RunMetadata | None):
        self.outputs = outputs
        self.metadata = metadata


class VariableStore(dict):
    """A session's variables; ``version`` increases on every write, so compiled plans
    (which fold variables into their weights) know when they went stale."""

    version = 0

    def __setitem__(self, k, v):
        super().__setitem__(k, v)
        self.version += 1

    def touch(self) -> None:
        """Records an in-place write (``copy_`` into an existing variable buffer)."""
        self.version += 1


class Session:
    def __init__(self, graph: Graph, device: str | torch.device | None = None):
        from .functions import has_functional_ops, lower_functional_ops

        # function calls / functional If / While (GraphDef.library) run as plain dataflow
        self.graph = lower_functional_ops(graph) if has_functional_ops(graph) else graph
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.variables: VariableStore = VariableStore()
        self._const_cache: dict = {}
        self._plans: dict = {}
        self._lock = threading.RLock()
        self._closed = False

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        self._closed = True
        self.variables.clear()
        self._const_cache.clear()
        self._plans.clear()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def runner(self) -> "Runner":
        return Runner(self)

    # ------------------------------------------------------------------ planning
    def _plan(self, feeds: Sequence[TensorName], fetch_nodes: Sequence[str], targets: Sequence[str]) -> _Plan:
        key = (tuple(sorted(str(f) for f in feeds)), tuple(fetch_nodes), tuple(targets))
        p = self._plans.get(key)
        if p is not None:
            return p
        fed_nodes = frozenset(f.name for f in feeds)
        needed: set[str] = set()
        stack = list(fetch_nodes) + list(targets)
        while stack:
            n = stack.pop()
            if n in needed:
                continue
            if n not in self.graph.nodes:
                raise KeyError(f"no node named {n!r} in graph")
            needed.add(n)
            if n in fed_nodes:
                continue
            node = self.graph.nodes[n]
            for src, _ in node.inputs:
                stack.append(src)
            stack.extend(node.control_inputs)
        order = self.graph.topo_order(needed)
        p = _Plan(order, fed_nodes, control_flow.plan_has_control_flow(self.graph, order))
        self._plans[key] = p
        return p

    # ------------------------------------------------------------------ execution
    def run(self, fetches: Sequence[str] | str = (), feed_dict: Mapping[str, Any] | None = None,
            targets: Sequence[str] = (), run_metadata: bool = False):
        """Executes the graph.  Returns a list of fetched values (or a single value if
        ``fetches`` is a string); with ``run_metadata=True`` returns a :class:`Run`."""
        if self._closed:
            raise RuntimeError("Session is closed")
        single = isinstance(fetches, str)
        fetch_list = [fetches] if single else list(fetches)
        feeds = {}
        for k, v in (feed_dict or {}).items():
            tn = TensorName.parse(k) if isinstance(k, str) else k
            feeds[(tn.name, tn.index)] = as_tensor(v, device=self.device) if not isinstance(v, StringTensor) else v
        fetch_names = [TensorName.parse(f) for f in fetch_list]
        target_names = [t.lstrip("^") for t in targets]
        with self._lock:
            plan = self._plan([TensorName(n, i) for n, i in feeds], [f.name for f in fetch_names], target_names)
            values: dict[tuple[str, int], Any] = dict(feeds)
            ctx = OpContext(self, self.device)
            stats = [] if run_metadata else None
            if plan.control_flow:
                values = control_flow.run_dataflow(self, plan, values, ctx, stats, lookup, ops_core.VarRef)
            for name in ([] if plan.control_flow else plan.order):
                if name in plan.fed_nodes:
                    continue
                node = self.graph.nodes[name]
                args = []
                deref = node.op not in REF_INPUT_OPS
                for i, (src, k) in enumerate(node.inputs):
                    try:
                        v = values[(src, k)]
                    except KeyError:
                        raise RuntimeError(f"input {src}:{k} of {name} was not computed") from None
                    if isinstance(v, ops_core.VarRef) and not v.resource and (deref or i > 0):
                        v = v.read()
                    args.append(v)
                fn = lookup(node.op)
                t0 = time.perf_counter_ns() if stats is not None else 0
                try:
                    outs = fn(ctx, node, *args)
                except (ValueError, TypeError, KeyError, RuntimeError, NotImplementedError) as e:
                    raise type(e)(f"{e} [node {name} ({node.op})]") from e
                if stats is not None:
                    if self.device.type == "cuda":
                        torch.cuda.synchronize(self.device)
                    t1 = time.perf_counter_ns()
                    stats.append(NodeExecStats(node_name=name, all_start_micros=t0 // 1000,
                                               op_end_rel_micros=(t1 - t0) // 1000,
                                               all_end_rel_micros=(t1 - t0) // 1000, timeline_label=node.op))
                for k, o in enumerate(outs):
                    values[(name, k)] = o
            result = []
            for f in fetch_names:
                try:
                    v = values[(f.name, f.index)]
                except KeyError:
                    if values.get((f.name, -1)) is control_flow.DEAD:
                        raise RuntimeError(f"fetch {f} is dead: it lies in a branch the run did not take") from None
                    raise KeyError(f"fetch {f} was not produced (node has {self._num_outputs(f.name)} outputs)") from None
                if v is control_flow.DEAD:
                    raise RuntimeError(f"fetch {f} is dead: it lies in a branch the run did not take")
                if isinstance(v, ops_core.VarRef):
                    v = v.read()
                result.append(v)
        out = result[0] if single else result
        if run_metadata:
            md = RunMetadata(step_stats=StepStats(dev_stats=[DeviceStepStats(device=str(self.device), node_stats=stats)]))
            return Run(out, md)
        return out

    def _num_outputs(self, name):
        return "?"

    # ------------------------------------------------------------------ helpers
    def initialize_variables(self, init_op: str | None = None):
        """Runs ``init_op`` or every ``*/Assign`` fed by an ``initial_value``."""
        if init_op is not None:
            self.run(targets=[init_op])
            return
        assigns = [n.name for n in self.graph.nodes.values() if n.op == "Assign" and n.inputs
                   and self.graph.nodes[n.inputs[0][0]].op in ("VariableV2", "Variable")]
        if assigns:
            self.run(targets=assigns)

    def variable_names(self) -> list[str]:
        return [n.name for n in self.graph.nodes.values() if n.op in ("VariableV2", "Variable", "VarHandleOp")]


class Runner:
    """Builder-style runner (TF Java ``Session.Runner``) used by ``ModelFunction``."""

    def __init__(self, session: Session):
        self.session = session
        self._feeds: dict[str, Any] = {}
        self._fetches: list[str] = []
        self._targets: list[str] = []

    def feed(self, name: str, index_or_value, value=None) -> "Runner":
        if value is None:
            self._feeds[name if ":" in name else f"{name}:0"] = index_or_value
        else:
            self._feeds[f"{name}:{index_or_value}"] = value
        return self

    def fetch(self, name: str, index: int | None = None) -> "Runner":
        self._fetches.append(name if index is None and ":" in name else f"{name}:{index or 0}")
        return self

    def add_target(self, name: str) -> "Runner":
        self._targets.append(name)
        return self

    def run(self) -> list:
        return self.session.run(self._fetches, self._feeds, self._targets)

    def run_and_fetch_metadata(self) -> Run:
        return self.session.run(self._fetches, self._feeds, self._targets, run_metadata=True)

    # camelCase aliases for parity with the JVM API used by the reference
    addTarget = add_target
    runAndFetchMetadata = run_and_fetch_metadata
