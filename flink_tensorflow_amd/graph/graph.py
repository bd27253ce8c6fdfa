"""Graph IR built from a TF GraphDef.

Replaces libtensorflow's ``TF_GraphImportGraphDef`` (reached by the reference through
``Graph.importGraphDef`` in ``LIB/util/GraphUtils.java:38-39`` and ``TFS/Graphs.scala:13-14``).
Import supports a name prefix; unlike the reference's ``GraphDefGraphLoader`` the prefix
is honoured.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Iterable

from ..proto.messages import AttrValue, GraphDef, NodeDef, TensorProto, TensorShapeProto
from ..types.dtypes import DataType


def parse_input(s: str) -> tuple[str, int, bool]:
    """``"name"`` / ``"name:k"`` / ``"^name"`` → (node, output index, is_control)."""
    if s.startswith("^"):
        return s[1:], -1, True
    if ":" in s:
        n, k = s.rsplit(":", 1)
        return n, int(k), False
    return s, 0, False


@dataclass
class Node:
    name: str
    op: str
    inputs: list[tuple[str, int]]          # data inputs (node, output index)
    control_inputs: list[str]
    attrs: dict[str, AttrValue]
    device: str = ""
    def_: NodeDef | None = field(default=None, repr=False)

    # ------------------------------------------------------------------ attr helpers
    def attr(self, key: str, default=None):
        a = self.attrs.get(key)
        if a is None:
            return default
        v = a.value()
        if a.which == "type":
            return DataType(v)
        if a.which == "list" and a.list is not None and a.list.type:
            return [DataType(t) for t in a.list.type]
        if a.which == "s":
            return v.decode("utf-8", errors="surrogateescape") if isinstance(v, bytes) else v
        return v

    def attr_bytes(self, key: str, default=b"") -> bytes:
        a = self.attrs.get(key)
        return a.s if a is not None else default

    def has_attr(self, key: str) -> bool:
        return key in self.attrs

    def shape_attr(self, key: str):
        a = self.attrs.get(key)
        if a is None or a.shape is None:
            return None
        return a.shape.as_list()

    def tensor_attr(self, key: str) -> TensorProto | None:
        a = self.attrs.get(key)
        return None if a is None else a.tensor

    def to_node_def(self) -> NodeDef:
        inputs = [f"{n}:{i}" if i else n for n, i in self.inputs] + [f"^{c}" for c in self.control_inputs]
        return NodeDef(name=self.name, op=self.op, input=inputs, device=self.device, attr=dict(self.attrs))


class Graph:
    """A mutable set of nodes keyed by name."""

    def __init__(self):
        self.nodes: dict[str, Node] = {}
        self.versions = None
        self.library: dict = {}  # function name -> FunctionDef (GraphDef.library; graph/functions.py)
        self._consumers: dict[str, list[str]] | None = None

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_graph_def(cls, gd: GraphDef | bytes, prefix: str = "") -> "Graph":
        g = cls()
        g.import_graph_def(gd, prefix)
        return g

    def import_graph_def(self, gd: GraphDef | bytes, prefix: str = "",
                         input_map: dict[str, str] | None = None) -> None:
        """Imports ``gd`` under ``prefix``.  ``input_map`` rewires references to tensors of
        the imported graph (``"input:0"``) onto existing tensors of this graph
        (``"normalized:0"``), like ``tf.import_graph_def(input_map=...)``."""
        if isinstance(gd, (bytes, bytearray, memoryview)):
            gd = GraphDef.decode(bytes(gd))
        pfx = (prefix.rstrip("/") + "/") if prefix else ""
        imap = {}
        for k, v in (input_map or {}).items():
            kn, ki, _ = parse_input(k)
            vn, vi, _ = parse_input(v)
            imap[(kn, ki)] = (vn, vi)
        for nd in gd.node:
            data, ctrl = [], []
            for s in nd.input:
                n, k, is_ctrl = parse_input(s)
                if is_ctrl:
                    ctrl.append(pfx + n)
                elif (n, k) in imap:
                    data.append(imap[(n, k)])
                else:
                    data.append((pfx + n, k))
            name = pfx + nd.name
            if name in self.nodes:
                raise ValueError(f"duplicate node name {name!r} on import")
            self.nodes[name] = Node(name, nd.op, data, ctrl, dict(nd.attr), nd.device, nd)
        if gd.versions is not None:
            self.versions = gd.versions
        if gd.library is not None:
            for f in gd.library.function:
                self.library[f.signature.name] = f
        self._consumers = None

    def add_node(self, node: Node) -> Node:
        if node.name in self.nodes:
            raise ValueError(f"duplicate node {node.name!r}")
        self.nodes[node.name] = node
        self._consumers = None
        return node

    def to_graph_def(self) -> GraphDef:
        from ..proto.messages import FunctionDefLibrary

        lib = FunctionDefLibrary(function=list(self.library.values())) if self.library else None
        return GraphDef(node=[n.to_node_def() for n in self.nodes.values()], versions=self.versions, library=lib)

    # ------------------------------------------------------------------ queries
    def __contains__(self, name: str) -> bool:
        return name in self.nodes

    def __getitem__(self, name: str) -> Node:
        try:
            return self.nodes[name]
        except KeyError:
            raise KeyError(f"no node named {name!r} in graph") from None

    def operation(self, name: str) -> Node | None:
        return self.nodes.get(name)

    def consumers(self, name: str) -> list[str]:
        if self._consumers is None:
            c: dict[str, list[str]] = {}
            for n in self.nodes.values():
                for src, _ in n.inputs:
                    c.setdefault(src, []).append(n.name)
                for src in n.control_inputs:
                    c.setdefault(src, []).append(n.name)
            self._consumers = c
        return self._consumers.get(name, [])

    def ops(self) -> set[str]:
        return {n.op for n in self.nodes.values()}

    def topo_order(self, needed: Iterable[str]) -> list[str]:
        """Topological order of ``needed`` (inputs before consumers)."""
        needed = set(needed)
        order: list[str] = []
        state: dict[str, int] = {}
        for root in sorted(needed):
            if state.get(root):
                continue
            stack = [(root, False)]
            while stack:
                name, done = stack.pop()
                if done:
                    if state.get(name) != 2:
                        state[name] = 2
                        order.append(name)
                    continue
                st = state.get(name, 0)
                if st == 2:
                    continue
                if st == 1:
                    continue
                state[name] = 1
                stack.append((name, True))
                node = self.nodes[name]
                merge = node.op in ("Merge", "RefMerge")
                for dep in [s for s, _ in node.inputs] + node.control_inputs:
                    if merge and self.nodes[dep].op in ("NextIteration", "RefNextIteration"):
                        continue  # a loop's back edge: the Merge does not wait for it
                    if dep in needed and state.get(dep, 0) == 0:
                        stack.append((dep, False))
                    elif dep in needed and state.get(dep) == 1 and not _is_loop_edge(self, dep, name):
                        raise ValueError(f"cycle in graph at {dep!r} -> {name!r}")
        return order


def _is_loop_edge(g: Graph, src: str, dst: str) -> bool:
    return g.nodes[dst].op in ("Merge", "NextIteration") or g.nodes[src].op == "NextIteration"


def make_attr(value=None, *, type=None, shape=None, tensor=None, list_=None, s=None, b=None, i=None, f=None) -> AttrValue:
    """Convenience constructor for AttrValue oneofs."""
    if type is not None:
        return AttrValue(type=int(DataType.of(type)))
    if shape is not None:
        return AttrValue(shape=TensorShapeProto.of(shape))
    if tensor is not None:
        return AttrValue(tensor=tensor)
    if list_ is not None:
        return AttrValue(list=list_)
    if s is not None:
        return AttrValue(s=s.encode() if isinstance(s, str) else s)
    if b is not None:
        return AttrValue(b=bool(b))
    if i is not None:
        return AttrValue(i=int(i))
    if f is not None:
        return AttrValue(f=float(f))
    raise ValueError("empty attr")
