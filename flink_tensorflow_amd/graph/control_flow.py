"""TF1 dataflow control flow: ``Switch`` / ``Merge`` / ``Enter`` / ``Exit`` /
``NextIteration`` / ``LoopCond`` (and the ``Ref*`` variants, ``_SwitchN``).

The reference runs any GraphDef through libtensorflow (``LIB/util/GraphUtils.java:31-41``,
``LIB/models/ModelFunction.scala:44-66``), and exported TF1 graphs use these ops for every
``tf.cond`` (``is_training`` switches around BatchNorm / dropout) and ``tf.while_loop``.
Two pieces here:

* ``run_dataflow`` — the interpreter's executor for plans that contain control flow:
  tagged-token dataflow in the style of TF's own executor.  Every value carries a tag
  ``(frame instance, iteration)``; ``Enter`` moves a value into a child frame (iteration 0),
  ``NextIteration`` into the next iteration, ``Exit`` back to the parent frame.  The branch
  ``Switch`` does not take emits a *dead* token; any op with a dead input (or dead control
  input) is dead, except ``Merge``, which forwards the first live input (or is dead when
  every input it waits for is dead: at iteration 0 its forward inputs, later its back
  edges).  Loop invariants (``Enter(is_constant=True)``) and input-less nodes of a frame
  are re-delivered to every iteration.  A dead ``NextIteration`` ends its loop; a dead
  ``Exit`` is held back and only propagates if the frame never produced a live one.
* ``fold_static_control_flow`` — the compiler's pre-pass: a ``Switch`` whose predicate is
  a compile-time constant (a ``Const``, or a ``PlaceholderWithDefault`` that is not fed,
  through ``Identity`` / ``LogicalNot`` / comparisons) is resolved, dead branches are
  dropped and single-live-input ``Merge``s become aliases, so an exported
  ``is_training``-gated CNN lowers to the same plan as its cond-free twin.

TF2 functional control flow (``If`` / ``While`` over a ``FunctionDefLibrary``) is not
handled here.
"""
from __future__ import annotations

import time
from collections import deque
from typing import Any

import torch

from .graph import Graph, Node
from .op_registry import REF_INPUT_OPS, register

SWITCH_OPS = {"Switch", "RefSwitch"}
MERGE_OPS = {"Merge", "RefMerge"}
ENTER_OPS = {"Enter", "RefEnter"}
EXIT_OPS = {"Exit", "RefExit"}
NEXT_OPS = {"NextIteration", "RefNextIteration"}
CONTROL_FLOW_OPS = SWITCH_OPS | MERGE_OPS | ENTER_OPS | EXIT_OPS | NEXT_OPS | {"LoopCond", "_SwitchN"}

REF_INPUT_OPS.update({"RefSwitch", "RefEnter", "RefExit", "RefNextIteration", "RefMerge", "RefIdentity"})


class _DeadType:
    __slots__ = ()

    def __repr__(self):
        return "<dead>"


DEAD = _DeadType()


def _pred(v) -> bool:
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise ValueError(f"control-flow predicate must be a scalar, got shape {tuple(v.shape)}")
        return bool(v.reshape(()).item())
    return bool(v)


# the interpreter reaches these only through ``run_dataflow``; registered so that the op
# set is known (``supported_ops``) and a plain walk over a graph without frames works
@register("Switch", "RefSwitch")
def _switch(ctx, node, data, pred):
    return (DEAD, data) if _pred(pred) else (data, DEAD)


@register("Merge", "RefMerge")
def _merge(ctx, node, *inputs):
    for i, v in enumerate(inputs):
        if v is not DEAD:
            return v, torch.tensor(i, dtype=torch.int32)
    return DEAD, DEAD


@register("Enter", "RefEnter", "Exit", "RefExit", "NextIteration", "RefNextIteration", "LoopCond")
def _forward(ctx, node, x):
    return (x,)


@register("_SwitchN")
def _switch_n(ctx, node, data, index):
    n = int(node.attr("num_outs", 0))
    k = int(index.reshape(()).item()) if isinstance(index, torch.Tensor) else int(index)
    if not 0 <= k < n:
        k = n - 1  # TF: an out-of-range index takes the last output
    return tuple(data if i == k else DEAD for i in range(n))


def plan_has_control_flow(graph: Graph, names) -> bool:
    return any(graph.nodes[n].op in CONTROL_FLOW_OPS for n in names)


# ------------------------------------------------------------------ static analysis
class _Topology:
    """Per-plan edge lists and static frames (cached on the session's plan)."""

    def __init__(self, graph: Graph, order: list[str], fed: frozenset):
        self.graph = graph
        needed = set(order)
        self.edges: dict[str, list[tuple[int, str, int]]] = {n: [] for n in order}
        for n in order:
            if n in fed:
                continue
            node = graph.nodes[n]
            for i, (src, k) in enumerate(node.inputs):
                self.edges.setdefault(src, []).append((k, n, i))
            for c in node.control_inputs:
                self.edges.setdefault(c, []).append((-1, n, -1))
        # Merge inputs that are loop back edges (from NextIteration): awaited from iteration 1 on
        self.back: dict[str, set[int]] = {}
        for n in order:
            node = graph.nodes[n]
            if node.op in MERGE_OPS and n not in fed:
                self.back[n] = {i for i, (s, _) in enumerate(node.inputs) if graph.nodes[s].op in NEXT_OPS}
        # static frame (tuple of frame names) of every node, for input-less nodes
        frame: dict[str, tuple | None] = {}
        for n in order:
            node = graph.nodes[n]
            srcs = [s for s, _ in node.inputs] + list(node.control_inputs)
            known = [frame[s] for s in srcs if s in frame and frame[s] is not None]
            if n in fed or not srcs:
                frame[n] = () if n in fed else None
                continue
            src_f = frame.get(node.inputs[0][0]) if node.inputs else None
            base = src_f if src_f is not None else (known[0] if known else ())
            if node.op in ENTER_OPS:
                frame[n] = base + (node.attr("frame_name", ""),)
            elif node.op in EXIT_OPS:
                frame[n] = base[:-1]
            else:
                frame[n] = base
        def input_frame(d):  # the frame a node reads its inputs in
            f = frame.get(d)
            if f is None or graph.nodes[d].op in EXIT_OPS:
                return None  # an Exit reads in its child frame: not derivable here
            return f[:-1] if graph.nodes[d].op in ENTER_OPS else f

        for n in order:  # input-less nodes take their consumers' frame (TF gives them a pivot edge)
            if frame[n] is None:
                fs = {input_frame(d) for _, d, _ in self.edges.get(n, [])} - {None}
                frame[n] = fs.pop() if len(fs) == 1 else ()
        self.sourceless: dict[tuple, list[str]] = {}
        for n in order:
            node = graph.nodes[n]
            if n not in fed and not node.inputs and not node.control_inputs:
                self.sourceless.setdefault(frame[n], []).append(n)
        self.needed = needed


class _Frame:
    __slots__ = ("static", "parent_tag", "invariants", "iters")

    def __init__(self, static: tuple, parent_tag):
        self.static = static
        self.parent_tag = parent_tag
        self.invariants: list[tuple[str, Any]] = []  # (constant Enter node, value)
        self.iters: set[int] = set()


class _Inst:
    __slots__ = ("inputs", "nrecv", "nctrl", "dead", "fired", "ndead")

    def __init__(self, n: int):
        self.inputs = [None] * n
        self.nrecv = 0
        self.nctrl = 0
        self.dead = False
        self.fired = False
        self.ndead = 0


_MISSING = object()


def run_dataflow(session, plan, feeds: dict, ctx, stats: list | None, lookup, var_ref_type) -> dict:
    """Executes ``plan`` (pruned node list) with control flow; returns the root-frame values
    ``{(node, output): value}`` (dead tensors as ``DEAD``)."""
    graph = session.graph
    topo = getattr(plan, "topology", None)
    if topo is None:
        topo = plan.topology = _Topology(graph, plan.order, plan.fed_nodes)
    edges, back = topo.edges, topo.back
    frames: dict[int, _Frame] = {0: _Frame((), None)}
    frames[0].iters.add(0)
    child_of: dict[tuple, int] = {}
    insts: dict[tuple, _Inst] = {}
    ready: deque = deque()
    root_vals: dict[tuple[str, int], Any] = dict(feeds)
    dead_exits: dict[tuple, bool] = {}  # (exit node, parent tag) -> went live
    ROOT = (0, 0)

    def start_iteration(fid: int, it: int):
        fr = frames[fid]
        if it in fr.iters:
            return
        fr.iters.add(it)
        tag = (fid, it)
        for enter, v in fr.invariants:
            send(enter, tag, (v,))
        for n in topo.sourceless.get(fr.static, ()):
            ready.append((n, tag, None))

    def deliver(dst: str, idx: int, tag, v):
        node = graph.nodes[dst]
        key = (dst, tag)
        st = insts.get(key)
        if st is None:
            st = insts[key] = _Inst(len(node.inputs))
        if st.fired:
            return  # a Merge that already forwarded a live input ignores the rest
        if node.op in MERGE_OPS:
            if idx < 0:
                return  # control inputs do not gate a Merge
            if v is not DEAD:
                st.fired = True
                ready.append((dst, tag, (v, idx)))
                return
            st.ndead += 1
            nb = len(back.get(dst, ()))
            # a loop Merge (NextIteration inputs) hears only its Enter inputs at iteration 0
            # and only its back edges after; any other Merge — a cond's Merge inside a loop
            # body included — waits for ALL its inputs to be dead, at every iteration
            if nb == 0:
                want = len(node.inputs)
            else:
                want = (len(node.inputs) - nb) if tag[1] == 0 else nb
            if st.ndead >= want:
                st.fired = True
                ready.append((dst, tag, DEAD))
            return
        if idx < 0:
            st.nctrl += 1
        else:
            st.inputs[idx] = v
            st.nrecv += 1
        if v is DEAD:
            st.dead = True
        if st.nrecv == len(node.inputs) and st.nctrl == len(node.control_inputs):
            st.fired = True
            ready.append((dst, tag, None))

    def send(src: str, tag, outs):
        """Delivers ``src``'s outputs (a tuple, or DEAD for all) along its edges."""
        for k, dst, i in edges.get(src, ()):
            if k < 0:
                v = DEAD if outs is DEAD else True
            else:
                v = DEAD if outs is DEAD else (outs[k] if k < len(outs) else _MISSING)
                if v is _MISSING:
                    raise RuntimeError(f"input {src}:{k} of {dst} was not computed")
            deliver(dst, i, tag, v)

    # fed tensors and input-less root nodes start the run
    for n in plan.fed_nodes:
        if n not in topo.needed:
            continue
        for k, dst, i in edges.get(n, ()):
            if k < 0:
                deliver(dst, i, ROOT, True)
            elif (n, k) in feeds:
                deliver(dst, i, ROOT, feeds[(n, k)])
            else:
                raise RuntimeError(f"input {n}:{k} of {dst} was not computed")
    for n in topo.sourceless.get((), ()):
        ready.append((n, ROOT, None))

    while True:
        while ready:
            name, tag, payload = ready.popleft()
            node = graph.nodes[name]
            op = node.op
            out_tag = tag
            # a fired Merge stays registered: its later (dead) inputs must find it fired
            st = insts.get((name, tag)) if op in MERGE_OPS else insts.pop((name, tag), None)
            t0 = time.perf_counter_ns() if stats is not None else 0
            if op in MERGE_OPS:
                outs = DEAD if payload is DEAD else (payload[0], torch.tensor(payload[1], dtype=torch.int32))
            elif st is not None and st.dead:
                outs = DEAD
            else:
                args = st.inputs if st is not None else []
                deref = op not in REF_INPUT_OPS
                args = [a.read() if isinstance(a, var_ref_type) and not a.resource and (deref or i > 0) else a
                        for i, a in enumerate(args)]
                try:
                    outs = tuple(lookup(op)(ctx, node, *args))
                except (ValueError, TypeError, KeyError, RuntimeError, NotImplementedError) as e:
                    raise type(e)(f"{e} [node {name} ({op})]") from e
            if op in ENTER_OPS:
                key = (tag, node.attr("frame_name", ""))
                fid = child_of.get(key)
                if fid is None:
                    fid = child_of[key] = len(frames)
                    frames[fid] = _Frame(frames[tag[0]].static + (key[1],), tag)
                out_tag = (fid, 0)
                start_iteration(fid, 0)
                if node.attr("is_constant", False) and outs is not DEAD:
                    fr = frames[fid]
                    fr.invariants.append((name, outs[0]))
                    for it in sorted(fr.iters):  # iterations that already started
                        send(name, (fid, it), outs)
                    continue
            elif op in EXIT_OPS:
                out_tag = frames[tag[0]].parent_tag
                if outs is DEAD:
                    dead_exits.setdefault((name, out_tag), False)
                    continue
                dead_exits[(name, out_tag)] = True
            elif op in NEXT_OPS:
                if outs is DEAD:
                    continue  # the loop ends here
                out_tag = (tag[0], tag[1] + 1)
                start_iteration(*out_tag)
            if stats is not None:
                from ..proto.messages import NodeExecStats

                t1 = time.perf_counter_ns()
                stats.append(NodeExecStats(node_name=name, all_start_micros=t0 // 1000,
                                           op_end_rel_micros=(t1 - t0) // 1000, all_end_rel_micros=(t1 - t0) // 1000,
                                           timeline_label=op))
            if out_tag == ROOT:
                if outs is DEAD:
                    root_vals[(name, -1)] = DEAD
                else:
                    for k, o in enumerate(outs):
                        root_vals[(name, k)] = o
            send(name, out_tag, outs)
        # quiescent: exits that never went live propagate their deadness (a loop inside an
        # untaken branch); anything they wake runs in the next pass
        pending = [k for k, live in dead_exits.items() if not live]
        if not pending:
            break
        for key in pending:
            dead_exits[key] = True
            send(key[0], key[1], DEAD)
    return root_vals


# ------------------------------------------------------------------ compile-time folding
_PRED_OPS = {"Const", "Identity", "LogicalNot", "LogicalAnd", "LogicalOr", "Equal", "NotEqual", "Less", "LessEqual",
             "Greater", "GreaterEqual", "Cast", "PlaceholderWithDefault", "Snapshot", "StopGradient", "Squeeze",
             "Reshape"}


def _static_value(graph: Graph, tensor: tuple[str, int], fed: set[str], memo: dict):
    """The value of ``tensor`` if it is a compile-time constant (its cone holds only
    constants and un-fed ``PlaceholderWithDefault``s), else None."""
    name, k = tensor
    if name in memo:
        return memo[name][k] if memo[name] is not None else None
    node = graph.nodes.get(name)
    if node is None or name in fed or node.op not in _PRED_OPS or node.control_inputs:
        memo[name] = None
        return None
    from .op_registry import OpContext, lookup

    args = []
    for src in node.inputs:
        v = _static_value(graph, src, fed, memo)
        if v is None:
            memo[name] = None
            return None
        args.append(v)

    class _S:  # a throw-away session for Const's cache
        _const_cache: dict = {}
        variables: dict = {}

    try:
        outs = tuple(lookup(node.op)(OpContext(_S(), torch.device("cpu")), node, *args))
    except Exception:  # noqa: BLE001 - not foldable: keep the Switch
        memo[name] = None
        return None
    memo[name] = outs
    return outs[k]


def fold_static_control_flow(graph: Graph, fed_tensors=(), fetches=()) -> Graph:
    """A copy of ``graph`` with every ``Switch`` on a compile-time-constant predicate
    resolved (returns ``graph`` itself when there is nothing to fold).  ``fed_tensors`` are
    the names the caller feeds (a fed ``PlaceholderWithDefault`` is not constant)."""
    from ..types.names import TensorName

    if not any(n.op in SWITCH_OPS for n in graph.nodes.values()):
        return graph
    fed = {TensorName.parse(f).name for f in fed_tensors}
    memo: dict = {}
    alias: dict[tuple[str, int], tuple[str, int]] = {}
    dead_t: set[tuple[str, int]] = set()
    folded: set[str] = set()
    for n in graph.nodes.values():
        if n.op not in SWITCH_OPS or len(n.inputs) != 2:
            continue
        pv = _static_value(graph, n.inputs[1], fed, memo)
        if pv is None:
            continue
        taken = 1 if _pred(pv) else 0
        alias[(n.name, taken)] = n.inputs[0]
        dead_t.add((n.name, 1 - taken))
        folded.add(n.name)
    if not folded:
        return graph

    def resolve(t):
        seen = 0
        while t in alias:
            t = alias[t]
            seen += 1
            if seen > len(alias):
                break
        return t

    dead_nodes: set[str] = set()
    const_nodes: dict[str, int] = {}  # Merge -> index of its live input (value_index becomes a Const)
    order = graph.topo_order(graph.nodes.keys())
    for name in order:
        if name in folded:
            continue
        node = graph.nodes[name]
        ins = [resolve(t) for t in node.inputs]
        is_dead = [t in dead_t or t[0] in dead_nodes for t in ins]
        if node.op in MERGE_OPS:
            live = [i for i, d in enumerate(is_dead) if not d]
            if not live:
                dead_nodes.add(name)
            elif len(live) == 1 and len(ins) > 1:
                alias[(name, 0)] = ins[live[0]]
                const_nodes[name] = live[0]
            continue
        if any(is_dead) or any(c in dead_nodes for c in node.control_inputs):
            dead_nodes.add(name)
    for f in fetches:
        t = TensorName.parse(f)
        if t.name in dead_nodes or (t.name, t.index) in dead_t:
            raise ValueError(f"fetch {f} lies in a branch that the constant predicate never takes")
    from .tensor_proto import make_tensor_proto
    from ..proto.messages import AttrValue
    from ..types.dtypes import DataType

    out = Graph()
    out.versions = graph.versions
    for name, node in graph.nodes.items():
        if name in dead_nodes or name in folded:
            continue
        if name in const_nodes:
            # the folded Merge: output 0 aliases its live input; output 1 (value_index) is a Const
            idx = torch.tensor(const_nodes[name], dtype=torch.int32)
            out.add_node(Node(name, "Const", [], [], {"value": AttrValue(tensor=make_tensor_proto(idx)),
                                                       "dtype": AttrValue(type=int(DataType.INT32))}))
            continue
        ins = []
        for t in node.inputs:
            r = resolve(t)
            if r[0] in const_nodes and r[1] == 1:
                r = (r[0], 0)  # value_index of a folded Merge: the Const node's output
            ins.append(r)
        ctrl = []
        for c in node.control_inputs:
            if c in folded:  # a control edge on a resolved Switch: wait for its data input instead
                src = graph.nodes[c].inputs[0][0]
                c = resolve((src, 0))[0] if (src, 0) in alias else src
            if c not in ctrl:
                ctrl.append(c)
        out.add_node(Node(name, node.op, ins, ctrl, dict(node.attrs), node.device, None))
    return out
