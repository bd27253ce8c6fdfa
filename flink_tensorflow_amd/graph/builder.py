"""``GraphBuilder``: emits TF GraphDefs from Python.

Covers the op DSL of the reference's ``EX/common/GraphBuilder.java:10-100`` (div, sub,
resizeBilinear, expandDims, cast, decodeJpeg, constant, variable, placeholder, build /
buildGraphDef) and extends it with the NN ops needed to express the model zoo
(ResNet-50, Inception-v3, MLPs) as real TF graphs that the executor imports and the
compiler lowers onto the CDNA4 kernels.

Every method returns the output tensor name (``"node:0"``); node names are uniquified
under an optional ``name_scope``.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from ..proto.messages import AttrListValue, AttrValue, GraphDef, NodeDef, TensorShapeProto, VersionDef
from ..types.dtypes import DataType
from ..types.tensor import as_tensor
from .graph import Graph
from .tensor_proto import make_tensor_proto


def _t(x) -> str:
    return x if ":" in x or x.startswith("^") else x


class GraphBuilder:
    def __init__(self):
        self.nodes: list[NodeDef] = []
        self._names: set[str] = set()
        self._scope: list[str] = []
        self.variables: dict[str, str] = {}  # var node name -> initializer Assign node

    # ------------------------------------------------------------------ naming
    @contextlib.contextmanager
    def name_scope(self, scope: str):
        self._scope.append(scope)
        try:
            yield
        finally:
            self._scope.pop()

    def _unique(self, base: str) -> str:
        name = "/".join(self._scope + [base]) if self._scope else base
        if name not in self._names:
            self._names.add(name)
            return name
        i = 1
        while f"{name}_{i}" in self._names:
            i += 1
        self._names.add(f"{name}_{i}")
        return f"{name}_{i}"

    def op(self, op_type: str, inputs=(), name: str | None = None, control=(), **attrs) -> str:
        nm = self._unique(name or op_type)
        ins = [_t(i) for i in inputs] + [f"^{c.split(':')[0]}" for c in control]
        nd = NodeDef(name=nm, op=op_type, input=ins, attr={k: _attr(v) for k, v in attrs.items() if v is not None})
        self.nodes.append(nd)
        return f"{nm}:0"

    # ------------------------------------------------------------------ reference DSL
    def constant(self, name: str, value, dtype=None) -> str:
        t = as_tensor(value if not isinstance(value, np.ndarray) else value, dtype=dtype)
        tp = make_tensor_proto(t)
        return self.op("Const", name=name, value=AttrValue(tensor=tp), dtype=DataType(tp.dtype))

    def placeholder(self, name: str, dtype, shape=None) -> str:
        return self.op("Placeholder", name=name, dtype=DataType.of(dtype),
                       shape=TensorShapeProto.of(shape) if shape is not None else TensorShapeProto(unknown_rank=True))

    def variable(self, name: str, dtype, shape) -> str:
        return self.op("VariableV2", name=name, dtype=DataType.of(dtype), shape=TensorShapeProto.of(shape),
                       container=b"", shared_name=b"")

    def variable_with_init(self, name: str, value) -> str:
        t = as_tensor(value)
        init = self.constant(f"{name}/initial_value", t)
        v = self.variable(name, DataType.of(t.dtype if isinstance(t, torch.Tensor) else DataType.STRING), tuple(t.shape))
        asg = self.op("Assign", [v, init], name=f"{name}/Assign", validate_shape=True, use_locking=True)
        self.variables[v.split(":")[0]] = asg.split(":")[0]
        return self.op("Identity", [v], name=f"{name}/read")

    def div(self, x, y, name=None) -> str:
        return self.op("Div", [x, y], name=name)

    def sub(self, x, y, name=None) -> str:
        return self.op("Sub", [x, y], name=name)

    def add(self, x, y, name=None) -> str:
        return self.op("Add", [x, y], name=name)

    def mul(self, x, y, name=None) -> str:
        return self.op("Mul", [x, y], name=name)

    def resize_bilinear(self, images, size, name=None, align_corners=False) -> str:
        return self.op("ResizeBilinear", [images, size], name=name, align_corners=align_corners)

    def expand_dims(self, x, dim, name=None) -> str:
        return self.op("ExpandDims", [x, dim], name=name)

    def cast(self, x, dst, name=None) -> str:
        return self.op("Cast", [x], name=name, DstT=DataType.of(dst))

    def decode_jpeg(self, contents, channels=3, name=None) -> str:
        return self.op("DecodeJpeg", [contents], name=name, channels=channels)

    # ------------------------------------------------------------------ NN extensions
    def identity(self, x, name=None) -> str:
        return self.op("Identity", [x], name=name)

    def relu(self, x, name=None) -> str:
        return self.op("Relu", [x], name=name)

    def conv2d(self, x, w, strides=(1, 1), padding="SAME", name=None, dilations=(1, 1)) -> str:
        return self.op("Conv2D", [x, w], name=name, strides=[1, strides[0], strides[1], 1], padding=padding.encode(),
                       data_format=b"NHWC", dilations=[1, dilations[0], dilations[1], 1], use_cudnn_on_gpu=True)

    def fused_batch_norm(self, x, scale, offset, mean, var, epsilon=1e-3, name=None) -> str:
        return self.op("FusedBatchNormV3", [x, scale, offset, mean, var], name=name, epsilon=float(epsilon),
                       is_training=False, data_format=b"NHWC")

    def lrn(self, x, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5, name=None) -> str:
        return self.op("LRN", [x], name=name, depth_radius=int(depth_radius), bias=float(bias), alpha=float(alpha),
                       beta=float(beta))

    def max_pool(self, x, ksize, strides, padding="VALID", name=None) -> str:
        return self.op("MaxPool", [x], name=name, ksize=[1, ksize[0], ksize[1], 1],
                       strides=[1, strides[0], strides[1], 1], padding=padding.encode(), data_format=b"NHWC")

    def avg_pool(self, x, ksize, strides, padding="VALID", name=None) -> str:
        return self.op("AvgPool", [x], name=name, ksize=[1, ksize[0], ksize[1], 1],
                       strides=[1, strides[0], strides[1], 1], padding=padding.encode(), data_format=b"NHWC")

    def mean(self, x, axes, keep_dims=False, name=None) -> str:
        a = self.constant(f"{(name or 'Mean')}/reduction_indices", np.asarray(axes, dtype=np.int32))
        return self.op("Mean", [x, a], name=name, keep_dims=keep_dims)

    def matmul(self, a, b, transpose_a=False, transpose_b=False, name=None) -> str:
        return self.op("MatMul", [a, b], name=name, transpose_a=transpose_a, transpose_b=transpose_b)

    def bias_add(self, x, b, name=None) -> str:
        return self.op("BiasAdd", [x, b], name=name, data_format=b"NHWC")

    def softmax(self, x, name=None) -> str:
        return self.op("Softmax", [x], name=name)

    def reshape(self, x, shape, name=None) -> str:
        s = self.constant(f"{(name or 'Reshape')}/shape", np.asarray(shape, dtype=np.int32))
        return self.op("Reshape", [x, s], name=name)

    def concat(self, xs, axis, name=None) -> str:
        a = self.constant(f"{(name or 'concat')}/axis", np.asarray(axis, dtype=np.int32))
        return self.op("ConcatV2", list(xs) + [a], name=name, N=len(xs))

    def top_k(self, x, k, name=None) -> str:
        kk = self.constant(f"{(name or 'TopKV2')}/k", np.asarray(k, dtype=np.int32))
        return self.op("TopKV2", [x, kk], name=name, sorted=True)

    def no_op(self, name, control=()) -> str:
        return self.op("NoOp", [], name=name, control=control)

    # ------------------------------------------------------------------ TF1 control flow
    def placeholder_with_default(self, default, name: str, shape=None) -> str:
        return self.op("PlaceholderWithDefault", [default], name=name, dtype=self._dtype_of(default),
                       shape=TensorShapeProto.of(shape) if shape is not None else TensorShapeProto(unknown_rank=True))

    def _dtype_of(self, t: str) -> DataType:
        nd = next(n for n in self.nodes if n.name == t.split(":")[0])
        a = nd.attr.get("dtype") or nd.attr.get("T")
        return DataType(a.type) if a is not None else DataType.FLOAT

    def _guard_new_nodes(self, start: int, pivot: str):
        """Input-less nodes made inside a branch / loop body get a control edge on the pivot
        (as TF's CondContext / WhileContext add), so they live in its frame and die with it."""
        p = "^" + pivot.split(":")[0]
        for nd in self.nodes[start:]:
            if not nd.input:
                nd.input.append(p)

    def cond(self, pred: str, true_fn, false_fn, inputs=(), name: str = "cond") -> str:
        """``tf.cond`` as TF1 emits it: ``Switch`` every input on ``pred``, build each branch
        on its Switch output, ``Merge`` the two results (output 0).  ``true_fn`` / ``false_fn``
        take the switched inputs and return one tensor."""
        with self.name_scope(name):
            sw = self.op("Switch", [pred, pred], name="Switch")
            swn = sw.split(":")[0]
            pivot_t = self.op("Identity", [f"{swn}:1"], name="switch_t")
            pivot_f = self.op("Identity", [f"{swn}:0"], name="switch_f")
            xs = [self.op("Switch", [x, pred], name="Switch").split(":")[0] for x in inputs]
            start = len(self.nodes)
            t = true_fn(*[f"{x}:1" for x in xs])
            self._guard_new_nodes(start, pivot_t)
            start = len(self.nodes)
            f = false_fn(*[f"{x}:0" for x in xs])
            self._guard_new_nodes(start, pivot_f)
            return self.op("Merge", [f, t], name="Merge", N=2)

    def while_loop(self, cond_fn, body_fn, loop_vars, invariants=(), name: str = "while") -> list[str]:
        """``tf.while_loop`` as TF1 emits it: ``Enter`` → ``Merge`` (with the back edge) →
        ``LoopCond`` → ``Switch``; the true side runs the body into ``NextIteration``, the
        false side leaves through ``Exit``.  ``invariants`` enter as loop constants.
        ``cond_fn`` / ``body_fn`` take (*loop vars, *invariants); returns the Exit tensors."""
        with self.name_scope(name):
            frame = "/".join(self._scope)
            enters = [self.op("Enter", [v], name="Enter", frame_name=frame, is_constant=False, parallel_iterations=10)
                      for v in loop_vars]
            invs = [self.op("Enter", [v], name="Enter", frame_name=frame, is_constant=True, parallel_iterations=10)
                    for v in invariants]
            merges = [self.op("Merge", [e, e], name="Merge", N=2) for e in enters]  # back edge patched below
            start = len(self.nodes)
            c = cond_fn(*merges, *invs)
            self._guard_new_nodes(start, merges[0])
            lc = self.op("LoopCond", [c], name="LoopCond")
            sws = [self.op("Switch", [m, lc], name="Switch").split(":")[0] for m in merges]
            exits = [self.op("Exit", [f"{sw}:0"], name="Exit") for sw in sws]
            body_in = [self.op("Identity", [f"{sw}:1"], name="Identity") for sw in sws]
            start = len(self.nodes)
            outs = body_fn(*body_in, *invs)
            outs = [outs] if isinstance(outs, str) else list(outs)
            self._guard_new_nodes(start, body_in[0])
            nexts = [self.op("NextIteration", [o], name="NextIteration") for o in outs]
            for m, nx in zip(merges, nexts):
                nd = next(n for n in self.nodes if n.name == m.split(":")[0])
                nd.input[1] = nx.split(":")[0]
            return exits

    # ------------------------------------------------------------------ output
    def build_graph_def(self) -> GraphDef:
        return GraphDef(node=list(self.nodes), versions=VersionDef(producer=26))

    buildGraphDef = build_graph_def

    def build(self, prefix: str = "") -> Graph:
        return Graph.from_graph_def(self.build_graph_def(), prefix)


def _attr(v) -> AttrValue:
    if isinstance(v, AttrValue):
        return v
    if isinstance(v, DataType):
        return AttrValue(type=int(v))
    if isinstance(v, TensorShapeProto):
        return AttrValue(shape=v)
    if isinstance(v, bool):
        return AttrValue(b=v)
    if isinstance(v, int):
        return AttrValue(i=v)
    if isinstance(v, float):
        return AttrValue(f=v)
    if isinstance(v, (bytes, str)):
        return AttrValue(s=v.encode() if isinstance(v, str) else v)
    if isinstance(v, (list, tuple)):
        if all(isinstance(e, DataType) for e in v) and v:
            return AttrValue(list=AttrListValue(type=[int(e) for e in v]))
        if all(isinstance(e, int) and not isinstance(e, bool) for e in v):
            return AttrValue(list=AttrListValue(i=list(v)))
        if all(isinstance(e, float) for e in v):
            return AttrValue(list=AttrListValue(f=list(v)))
        if all(isinstance(e, (bytes, str)) for e in v):
            return AttrValue(list=AttrListValue(s=[e.encode() if isinstance(e, str) else e for e in v]))
        if all(isinstance(e, TensorShapeProto) for e in v):
            return AttrValue(list=AttrListValue(shape=list(v)))
    raise TypeError(f"cannot convert {v!r} to an AttrValue")
