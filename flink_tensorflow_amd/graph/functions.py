"""Function calls and functional control flow in GraphDefs (``GraphDef.library``).

The reference hands any GraphDef to libtensorflow (``LIB/util/GraphUtils.java:31-41``).
Graphs written with TF's control flow v2 — and every TF2-style signature, which wraps its
body in ``StatefulPartitionedCall`` — carry a ``FunctionDefLibrary`` and call into it with
``PartitionedCall`` / ``StatefulPartitionedCall``, ``If`` / ``StatelessIf`` and ``While`` /
``StatelessWhile``.  ``lower_functional_ops`` rewrites them into plain dataflow, the way
TF's own ``LowerFunctionalOpsPass`` does before execution:

* a call is inlined: the body's nodes are copied under the call's name as a prefix, its
  arguments wired to the call's inputs, and every consumer of the call's outputs rewired
  to the body's return values;
* ``If`` becomes ``Switch`` on every argument, both branches inlined on the two Switch
  sides (input-less branch nodes hang off a pivot so they die with their branch) and one
  ``Merge`` per output;
* ``While`` becomes the TF1 loop frame: ``Enter`` → ``Merge`` (back edge from
  ``NextIteration``) → the inlined condition → ``LoopCond`` → ``Switch`` → ``Exit`` /
  the inlined body → ``NextIteration``.

The result runs on the interpreter's dataflow executor (``graph/control_flow.py``), and
the compiler folds lowered ``If``s with a compile-time-constant predicate like TF1 conds.
The call node itself stays as an ``IdentityN`` over the return values (or Merges / Exits),
so signatures that fetch ``StatefulPartitionedCall:0`` keep working.

Inside a FunctionDef, inputs name a signature argument (``"x"``) or a node output as
``"node:out_arg:index"``; the flat output index needs the op's output-argument layout,
listed below for the multi-output ops (every other op has one output argument).
"""
from __future__ import annotations

from .graph import Graph, Node

CALL_OPS = {"PartitionedCall", "StatefulPartitionedCall"}
IF_OPS = {"If", "StatelessIf"}
WHILE_OPS = {"While", "StatelessWhile"}
FUNCTIONAL_OPS = CALL_OPS | IF_OPS | WHILE_OPS

# output argument names, in order, of ops with more than one output argument
_OUT_ARGS = {
    "Switch": ["output_false", "output_true"], "RefSwitch": ["output_false", "output_true"],
    "Merge": ["output", "value_index"], "RefMerge": ["output", "value_index"],
    "TopKV2": ["values", "indices"], "TopK": ["values", "indices"],
    "FusedBatchNorm": ["y", "batch_mean", "batch_variance", "reserve_space_1", "reserve_space_2"],
    "FusedBatchNormV2": ["y", "batch_mean", "batch_variance", "reserve_space_1", "reserve_space_2"],
    "FusedBatchNormV3": ["y", "batch_mean", "batch_variance", "reserve_space_1", "reserve_space_2",
                         "reserve_space_3"],
    "Unique": ["y", "idx"], "UniqueWithCounts": ["y", "idx", "count"],
    "SoftmaxCrossEntropyWithLogits": ["loss", "backprop"],
    "SparseSoftmaxCrossEntropyWithLogits": ["loss", "backprop"],
}

_MAX_DEPTH = 64


def has_functional_ops(graph: Graph) -> bool:
    return any(n.op in FUNCTIONAL_OPS for n in graph.nodes.values())


def _func(node: Node, key: str):
    a = node.attrs.get(key)
    if a is None or a.func is None or not a.func.name:
        raise ValueError(f"{node.op} {node.name}: missing function attr {key!r}")
    return a.func.name, dict(a.func.attr)


class _Lowering:
    def __init__(self, graph: Graph):
        self.src = graph
        self.lib = graph.library
        self.out = Graph()
        self.out.versions = graph.versions
        self.out.library = dict(graph.library)
        self.remap: dict[tuple[str, int], tuple[str, int]] = {}

    # ------------------------------------------------------------------ helpers
    def _add(self, name, op, inputs=(), ctrl=(), attrs=None) -> str:
        self.out.add_node(Node(name, op, list(inputs), list(ctrl), dict(attrs or {})))
        return name

    def _fdef(self, name):
        f = self.lib.get(name)
        if f is None:
            raise ValueError(f"function {name!r} is not in the graph's library")
        return f

    def inline(self, prefix: str, fname: str, args: list, anchor: list[str], fattrs: dict | None = None):
        """Copies the body of ``fname`` under ``prefix``; returns (return tensors in
        output-argument order, control-return node names).  ``fattrs``: the instantiation
        attrs of the call (substituted for ``$name`` placeholders in the body)."""
        f = self._fdef(fname)
        fattrs = {**dict(f.attr), **(fattrs or {})}
        sig = f.signature
        if len(args) != len(sig.input_arg):
            raise ValueError(f"function {fname!r} takes {len(sig.input_arg)} arguments, got {len(args)}")
        argmap = {a.name: t for a, t in zip(sig.input_arg, args)}
        ops = {nd.name: nd.op for nd in f.node_def}

        def tensor(ref: str):
            parts = ref.split(":")
            if len(parts) == 1:
                if ref in argmap:
                    return argmap[ref]
                return (f"{prefix}/{ref}", 0)
            node = parts[0]
            if node in argmap and len(parts) == 2 and parts[1].isdigit():
                return argmap[node]
            if len(parts) == 2:
                return (f"{prefix}/{node}", int(parts[1]) if parts[1].isdigit() else 0)
            out_arg, idx = parts[1], int(parts[2])
            layout = _OUT_ARGS.get(ops.get(node, ""))
            flat = (layout.index(out_arg) if out_arg in layout else 0) + idx if layout else idx
            return (f"{prefix}/{node}", flat)

        for nd in f.node_def:
            data, ctrl = [], []
            for inp in nd.input:
                if inp.startswith("^"):
                    c = inp[1:]
                    if c not in argmap:
                        ctrl.append(f"{prefix}/{c}")
                else:
                    data.append(tensor(inp))
            if not data and not ctrl:
                ctrl = list(anchor)  # lives in the caller's frame / branch
            attrs = {k: (fattrs.get(v.placeholder, v) if getattr(v, "which", None) == "placeholder" else v)
                     for k, v in nd.attr.items()}
            self._add(f"{prefix}/{nd.name}", nd.op, data, ctrl, attrs)
        rets = []
        for a in sig.output_arg:
            r = f.ret.get(a.name)
            if r is None:
                raise ValueError(f"function {fname!r} does not return {a.name!r}")
            rets.append(tensor(r))
        cret = [f"{prefix}/{v.split(':')[0]}" for v in f.control_ret.values()]
        return rets, cret

    def _gate(self, n: Node, tensors: list) -> tuple[list, list[str]]:
        """TF's inliner semantics for a call / If / While with control inputs: one
        ``<name>/input_control`` NoOp carries them and every argument passes through an
        Identity that depends on it, so each inlined node that reads an argument (not only
        the input-less ones) waits for the caller's control dependencies, and pruning keeps
        them.  Returns (gated arguments, anchor for input-less body nodes)."""
        if not n.control_inputs:
            return list(tensors), []
        ic = self._add(f"{n.name}/input_control", "NoOp", [], list(n.control_inputs))
        gated = [(self._add(f"{n.name}/arg_{i}", "Identity", [t], [ic]), 0) for i, t in enumerate(tensors)]
        return gated, [ic]

    # ------------------------------------------------------------------ lowering
    def call(self, n: Node):
        fn, fa = _func(n, "f")
        args, anchor = self._gate(n, list(n.inputs))
        rets, cret = self.inline(n.name + "/body", fn, args, anchor, fa)
        for i, r in enumerate(rets):
            self.remap[(n.name, i)] = r
        self._add(n.name, "IdentityN", rets, cret)

    def if_(self, n: Node):
        gated, _ = self._gate(n, list(n.inputs))
        cond, args = gated[0], gated[1:]
        sw = self._add(f"{n.name}/switch_pred", "Switch", [cond, cond])
        pt = self._add(f"{n.name}/pivot_t", "Identity", [(sw, 1)])
        pf = self._add(f"{n.name}/pivot_f", "Identity", [(sw, 0)])
        sws = [self._add(f"{n.name}/switch_{i}", "Switch", [a, cond]) for i, a in enumerate(args)]
        tn, ta = _func(n, "then_branch")
        en, ea = _func(n, "else_branch")
        t_rets, _ = self.inline(f"{n.name}/then", tn, [(s, 1) for s in sws], [pt], ta)
        e_rets, _ = self.inline(f"{n.name}/else", en, [(s, 0) for s in sws], [pf], ea)
        if len(t_rets) != len(e_rets):
            raise ValueError(f"If {n.name}: branches return {len(t_rets)} and {len(e_rets)} values")
        merges = []
        for j, (e, t) in enumerate(zip(e_rets, t_rets)):
            m = self._add(f"{n.name}/merge_{j}", "Merge", [e, t])
            merges.append((m, 0))
            self.remap[(n.name, j)] = (m, 0)
        # (control returns of a branch are not joined: a node of the untaken branch is dead)
        self._add(n.name, "IdentityN", merges)

    def while_(self, n: Node):
        vars_, _ = self._gate(n, list(n.inputs))
        if not vars_:
            raise ValueError(f"While {n.name} has no loop variables")
        frame = n.name
        enters = [self._add(f"{n.name}/enter_{i}", "Enter", [v], [],
                            {"frame_name": _s_attr(frame), "is_constant": _b_attr(False),
                             "parallel_iterations": _i_attr(10)}) for i, v in enumerate(vars_)]
        merges = [self._add(f"{n.name}/merge_{i}", "Merge", [(e, 0), (e, 0)]) for i, e in enumerate(enters)]
        cn, ca = _func(n, "cond")
        (c,), _ = self.inline(f"{n.name}/cond", cn, [(m, 0) for m in merges], [merges[0]], ca)
        lc = self._add(f"{n.name}/loop_cond", "LoopCond", [c])
        sws = [self._add(f"{n.name}/switch_{i}", "Switch", [(m, 0), (lc, 0)]) for i, m in enumerate(merges)]
        exits = [self._add(f"{n.name}/exit_{i}", "Exit", [(s, 0)]) for i, s in enumerate(sws)]
        ids = [self._add(f"{n.name}/ident_{i}", "Identity", [(s, 1)]) for i, s in enumerate(sws)]
        bn, ba = _func(n, "body")
        b_rets, _ = self.inline(f"{n.name}/body", bn, [(x, 0) for x in ids], [ids[0]], ba)
        if len(b_rets) != len(vars_):
            raise ValueError(f"While {n.name}: body returns {len(b_rets)} values for {len(vars_)} loop variables")
        for i, (m, b) in enumerate(zip(merges, b_rets)):
            nx = self._add(f"{n.name}/next_{i}", "NextIteration", [b])
            self.out.nodes[m].inputs[1] = (nx, 0)
        for i, e in enumerate(exits):
            self.remap[(n.name, i)] = (e, 0)
        self._add(n.name, "IdentityN", [(e, 0) for e in exits])

    def run(self) -> Graph:
        for n in self.src.nodes.values():
            if n.op in CALL_OPS:
                self.call(n)
            elif n.op in IF_OPS:
                self.if_(n)
            elif n.op in WHILE_OPS:
                self.while_(n)
            else:
                self.out.add_node(Node(n.name, n.op, list(n.inputs), list(n.control_inputs), dict(n.attrs), n.device,
                                       n.def_))

        def resolve(t):
            seen = 0
            while t in self.remap and seen <= len(self.remap):
                t = self.remap[t]
                seen += 1
            return t

        for node in self.out.nodes.values():
            node.inputs = [resolve(t) for t in node.inputs]
        return self.out


def _s_attr(v: str):
    from ..proto.messages import AttrValue

    return AttrValue(s=v.encode())


def _b_attr(v: bool):
    from ..proto.messages import AttrValue

    return AttrValue(b=v)


def _i_attr(v: int):
    from ..proto.messages import AttrValue

    return AttrValue(i=v)


def lower_functional_ops(graph: Graph) -> Graph:
    """``graph`` with every function call / functional If / While lowered to plain
    dataflow (nested ones too); ``graph`` itself when it has none."""
    g = graph
    for _ in range(_MAX_DEPTH):
        if not has_functional_ops(g):
            return g
        g = _Lowering(g).run()
    raise ValueError(f"function calls nested deeper than {_MAX_DEPTH} levels (recursive functions?)")
