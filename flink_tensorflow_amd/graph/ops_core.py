"""Core TF op kernels: plumbing, variables, math, shape manipulation, reductions."""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ..types.dtypes import DataType
from ..types.tensor import StringTensor, dtype_of
from .op_registry import register
from .tensor_proto import tensor_from_proto


class FailedPreconditionError(RuntimeError):
    pass


class VarRef:
    """A reference to a session variable (the output of VariableV2 / VarHandleOp)."""

    __slots__ = ("session", "name", "dtype", "shape", "resource")

    def __init__(self, session, name, dtype, shape, resource: bool = False):
        self.session, self.name, self.dtype, self.shape = session, name, dtype, shape
        # a resource handle (VarHandleOp) is never read implicitly: only ReadVariableOp /
        # Assign*VariableOp / ResourceGather touch it; pass-through ops (Identity, function
        # arguments) forward the handle
        self.resource = resource

    def read(self):
        v = self.session.variables.get(self.name)
        if v is None:
            raise FailedPreconditionError(f"Attempting to use uninitialized value {self.name}")
        return v

    def write(self, value, validate_shape=True):
        cur = self.session.variables.get(self.name)
        if validate_shape and self.shape is not None and not isinstance(value, StringTensor):
            exp = tuple(self.shape)
            if -1 not in exp and tuple(value.shape) != exp:
                raise ValueError(f"Assign requires shapes to match: {self.name} {exp} vs {tuple(value.shape)}")
        if (cur is not None and isinstance(cur, torch.Tensor) and isinstance(value, torch.Tensor)
                and cur.shape == value.shape and cur.dtype == value.dtype and cur.device == value.device):
            cur.copy_(value)  # in-place: keeps buffers captured by compiled plans valid
            touch = getattr(self.session.variables, "touch", None)
            if touch is not None:
                touch()
            return cur
        v = value.clone() if isinstance(value, torch.Tensor) else value
        self.session.variables[self.name] = v
        return v


def _dev(ctx, t):
    return t.to(ctx.device) if isinstance(t, torch.Tensor) and t.device != ctx.device else t


# ------------------------------------------------------------------ plumbing
@register("Const")
def _const(ctx, node):
    key = ("const", node.name)
    cache = ctx.session._const_cache
    if key not in cache:
        t = tensor_from_proto(node.tensor_attr("value"))
        cache[key] = _dev(ctx, t)
    return (cache[key],)


@register("Placeholder", "PlaceholderV2")
def _placeholder(ctx, node):
    raise ValueError(f"You must feed a value for placeholder tensor '{node.name}'")


@register("PlaceholderWithDefault")
def _placeholder_default(ctx, node, x):
    return (x,)


@register("Identity", "StopGradient", "Snapshot", "PreventGradient", "CheckNumerics", "EnsureShape")
def _identity(ctx, node, x, *rest):
    return (x,)


@register("IdentityN")
def _identity_n(ctx, node, *xs):
    return tuple(xs)


@register("NoOp", "ControlTrigger")
def _noop(ctx, node, *xs):
    return ()


@register("Print", "PrintV2")
def _print(ctx, node, x, *data):
    print(node.attr("message", ""), [d.tolist() if hasattr(d, "tolist") else d for d in data])
    return (x,)


# ------------------------------------------------------------------ variables
@register("VariableV2", "Variable", "VarHandleOp")
def _variable(ctx, node):
    name = node.attr("shared_name") or node.name
    dt = node.attr("dtype")
    shape = node.shape_attr("shape")
    return (VarRef(ctx.session, name, dt, shape, resource=node.op == "VarHandleOp"),)


@register("Assign")
def _assign(ctx, node, ref, value):
    return (ref.write(_dev(ctx, value), validate_shape=node.attr("validate_shape", True)),)


@register("AssignAdd")
def _assign_add(ctx, node, ref, value):
    return (ref.write(ref.read() + value, False),)


@register("AssignSub")
def _assign_sub(ctx, node, ref, value):
    return (ref.write(ref.read() - value, False),)


@register("AssignVariableOp")
def _assign_var_op(ctx, node, ref, value):
    ref.write(_dev(ctx, value), validate_shape=False)
    return ()


@register("AssignAddVariableOp")
def _assign_add_var_op(ctx, node, ref, value):
    ref.write(ref.read() + value, False)
    return ()


@register("ReadVariableOp")
def _read_var(ctx, node, ref):
    return (ref.read(),)


@register("IsVariableInitialized")
def _is_init(ctx, node, ref):
    return (torch.tensor(ctx.session.variables.get(ref.name) is not None),)


@register("ScatterUpdate")
def _scatter_update(ctx, node, ref, idx, upd):
    v = ref.read().clone()
    v[idx.long()] = upd.to(v.dtype)
    return (ref.write(v, False),)


@register("ScatterAdd")
def _scatter_add(ctx, node, ref, idx, upd):
    v = ref.read().clone()
    v.index_add_(0, idx.long().reshape(-1), upd.reshape(-1, *v.shape[1:]).to(v.dtype))
    return (ref.write(v, False),)


# ------------------------------------------------------------------ elementwise math
def _binary(fn):
    def k(ctx, node, a, b):
        return (fn(a, b),)

    return k


def _same_dtype(a, b):
    return b.to(a.dtype) if isinstance(b, torch.Tensor) and b.dtype != a.dtype else b


register("Add", "AddV2")(lambda ctx, node, a, b: (_add(a, b),))


def _add(a, b):
    if isinstance(a, StringTensor):
        return StringTensor(np.char.add(a.array.astype(bytes), b.array.astype(bytes)).astype(object))
    return a + _same_dtype(a, b)


register("Sub")(_binary(lambda a, b: a - _same_dtype(a, b)))
register("Mul")(_binary(lambda a, b: a * _same_dtype(a, b)))
register("RealDiv")(_binary(lambda a, b: a / _same_dtype(a, b)))
register("Maximum")(_binary(lambda a, b: torch.maximum(a, _same_dtype(a, b))))
register("Minimum")(_binary(lambda a, b: torch.minimum(a, _same_dtype(a, b))))
register("Pow")(_binary(lambda a, b: torch.pow(a, _same_dtype(a, b))))
register("SquaredDifference")(_binary(lambda a, b: (a - _same_dtype(a, b)) ** 2))
register("Equal")(_binary(lambda a, b: a == b))
register("NotEqual")(_binary(lambda a, b: a != b))
register("Less")(_binary(lambda a, b: a < b))
register("LessEqual")(_binary(lambda a, b: a <= b))
register("Greater")(_binary(lambda a, b: a > b))
register("GreaterEqual")(_binary(lambda a, b: a >= b))
register("LogicalAnd")(_binary(lambda a, b: a & b))
register("LogicalOr")(_binary(lambda a, b: a | b))
register("BiasAdd", "BiasAddV1")(lambda ctx, node, x, b: (_bias_add(node, x, b),))


def _bias_add(node, x, b):
    if node.attr("data_format", "NHWC") == "NCHW" and x.dim() >= 3:
        return x + b.reshape(1, -1, *([1] * (x.dim() - 2)))
    return x + b


@register("Div")
def _div(ctx, node, a, b):
    if not a.is_floating_point():
        return (torch.div(a, b, rounding_mode="floor"),)
    return (a / _same_dtype(a, b),)


@register("FloorDiv")
def _floordiv(ctx, node, a, b):
    return (torch.div(a, b, rounding_mode="floor"),)


@register("FloorMod", "Mod")
def _mod(ctx, node, a, b):
    return (torch.remainder(a, b),)


def _unary(fn):
    def k(ctx, node, x):
        return (fn(x),)

    return k


register("Neg")(_unary(torch.neg))
register("Abs")(_unary(torch.abs))
register("Square")(_unary(lambda x: x * x))
register("Sqrt")(_unary(torch.sqrt))
register("Rsqrt")(_unary(torch.rsqrt))
register("Exp")(_unary(torch.exp))
register("Log")(_unary(torch.log))
register("Log1p")(_unary(torch.log1p))
register("Tanh")(_unary(torch.tanh))
register("Sigmoid")(_unary(torch.sigmoid))
register("Relu")(_unary(F.relu))
register("Relu6")(_unary(lambda x: torch.clamp(x, 0, 6)))
register("Elu")(_unary(F.elu))
register("Selu")(_unary(F.selu))
register("Softplus")(_unary(F.softplus))
register("Softsign")(_unary(F.softsign))
register("Erf")(_unary(torch.erf))
register("Floor")(_unary(torch.floor))
register("Ceil")(_unary(torch.ceil))
register("Round")(_unary(torch.round))
register("Sign")(_unary(torch.sign))
register("Reciprocal", "Inv")(_unary(torch.reciprocal))
register("LogicalNot")(_unary(torch.logical_not))
register("ZerosLike")(_unary(torch.zeros_like))
register("OnesLike")(_unary(torch.ones_like))
register("Gelu")(lambda ctx, node, x: (F.gelu(x, approximate="tanh" if node.attr("approximate", False) else "none"),))


@register("LeakyRelu")
def _leaky(ctx, node, x):
    return (F.leaky_relu(x, node.attr("alpha", 0.2)),)


@register("AddN")
def _addn(ctx, node, *xs):
    out = xs[0]
    for x in xs[1:]:
        out = out + x
    return (out,)


@register("Cast")
def _cast(ctx, node, x):
    dst = node.attr("DstT")
    if isinstance(x, StringTensor):
        raise TypeError("Cast from STRING is not supported")
    return (x.to(dst.torch),)


@register("Select", "SelectV2")
def _select(ctx, node, c, a, b):
    if node.op == "Select" and c.dim() == 1 and a.dim() > 1:
        c = c.reshape(-1, *([1] * (a.dim() - 1)))
    return (torch.where(c, a, b),)


@register("ClipByValue")
def _clip(ctx, node, x, lo, hi):
    return (torch.clamp(x, lo, hi),)


# ------------------------------------------------------------------ matmul family
@register("MatMul")
def _matmul(ctx, node, a, b):
    if node.attr("transpose_a", False):
        a = a.t()
    if node.attr("transpose_b", False):
        b = b.t()
    return (a @ b,)


@register("BatchMatMul", "BatchMatMulV2", "BatchMatMulV3")
def _bmm(ctx, node, a, b):
    if node.attr("adj_x", False):
        a = a.transpose(-1, -2)
    if node.attr("adj_y", False):
        b = b.transpose(-1, -2)
    return (torch.matmul(a, b),)


# ------------------------------------------------------------------ shapes
def _ints(t) -> list[int]:
    return [int(v) for v in (t.reshape(-1).tolist() if isinstance(t, torch.Tensor) else list(t))]


@register("Shape")
def _shape(ctx, node, x):
    dt = node.attr("out_type", DataType.INT32)
    return (torch.tensor(list(x.shape), dtype=dt.torch),)


@register("ShapeN")
def _shape_n(ctx, node, *xs):
    dt = node.attr("out_type", DataType.INT32)
    return tuple(torch.tensor(list(x.shape), dtype=dt.torch) for x in xs)


@register("Size")
def _size(ctx, node, x):
    return (torch.tensor(int(np.prod(x.shape)), dtype=node.attr("out_type", DataType.INT32).torch),)


@register("Rank")
def _rank(ctx, node, x):
    return (torch.tensor(len(x.shape), dtype=torch.int32),)


@register("Reshape")
def _reshape(ctx, node, x, shape):
    return (x.reshape(tuple(_ints(shape))),)


@register("Squeeze")
def _squeeze(ctx, node, x):
    dims = node.attr("squeeze_dims", []) or []
    if isinstance(x, StringTensor):
        return (StringTensor(np.squeeze(x.array, axis=tuple(dims) if dims else None)),)
    if not dims:
        return (x.squeeze(),)
    for d in sorted([d % x.dim() for d in dims], reverse=True):
        x = x.squeeze(d)
    return (x,)


@register("ExpandDims")
def _expand_dims(ctx, node, x, axis):
    a = _ints(axis)[0]
    if isinstance(x, StringTensor):
        return (StringTensor(np.expand_dims(x.array, a)),)
    if a < 0:
        a += x.dim() + 1
    return (x.unsqueeze(a),)


@register("Pack")
def _pack(ctx, node, *xs):
    axis = node.attr("axis", 0)
    if isinstance(xs[0], StringTensor):
        return (StringTensor(np.stack([x.array for x in xs], axis=axis)),)
    return (torch.stack(list(xs), dim=axis),)


@register("Unpack")
def _unpack(ctx, node, x):
    axis = node.attr("axis", 0)
    return tuple(torch.unbind(x, dim=axis))


@register("ConcatV2")
def _concat_v2(ctx, node, *args):
    *xs, axis = args
    a = _ints(axis)[0]
    if isinstance(xs[0], StringTensor):
        return (StringTensor(np.concatenate([x.array for x in xs], axis=a)),)
    return (torch.cat(list(xs), dim=a),)


@register("Concat")
def _concat(ctx, node, axis, *xs):
    return (torch.cat(list(xs), dim=_ints(axis)[0]),)


@register("Transpose")
def _transpose(ctx, node, x, perm):
    return (x.permute(*_ints(perm)).contiguous(),)


@register("Fill")
def _fill(ctx, node, dims, value):
    return (torch.full(tuple(_ints(dims)), value.item(), dtype=value.dtype, device=ctx.device),)


@register("Range")
def _range(ctx, node, start, limit, delta):
    dt = node.attr("Tidx", DataType.INT32)
    return (torch.arange(start.item(), limit.item(), delta.item(), dtype=dt.torch, device=ctx.device),)


@register("Tile")
def _tile(ctx, node, x, multiples):
    return (x.repeat(*_ints(multiples)),)


@register("Pad", "PadV2", "MirrorPad")
def _pad(ctx, node, x, paddings, *cv):
    p = np.asarray(_ints(paddings)).reshape(-1, 2)
    flat = []
    for lo, hi in p[::-1]:
        flat += [int(lo), int(hi)]
    if node.op == "MirrorPad":
        mode = "reflect" if node.attr("mode", "REFLECT") == "REFLECT" else "replicate"
        return (F.pad(x, flat, mode=mode),)
    value = cv[0].item() if cv else 0
    return (F.pad(x, flat, value=value),)


@register("Slice")
def _slice(ctx, node, x, begin, size):
    b, s = _ints(begin), _ints(size)
    idx = tuple(slice(bi, bi + si if si >= 0 else None) for bi, si in zip(b, s))
    return (x[idx],)


@register("StridedSlice")
def _strided_slice(ctx, node, x, begin, end, strides):
    b, e, s = _ints(begin), _ints(end), _ints(strides)
    bm, em = node.attr("begin_mask", 0), node.attr("end_mask", 0)
    ell, nam, sam = node.attr("ellipsis_mask", 0), node.attr("new_axis_mask", 0), node.attr("shrink_axis_mask", 0)
    idx = []
    squeeze = []
    for i in range(len(b)):
        if ell & (1 << i):
            idx.append(Ellipsis)
            continue
        if nam & (1 << i):
            idx.append(None)
            continue
        if sam & (1 << i):
            idx.append(b[i])
            continue
        lo = None if bm & (1 << i) else b[i]
        hi = None if em & (1 << i) else e[i]
        idx.append(slice(lo, hi, s[i]))
    if any(isinstance(i, slice) and i.step is not None and i.step < 0 for i in idx):
        # torch has no negative-step slicing: flip then slice
        arr = x.cpu().numpy() if isinstance(x, torch.Tensor) else x.array
        return (torch.from_numpy(np.ascontiguousarray(arr[tuple(idx)])).to(x.device),)
    del squeeze
    return (x[tuple(idx)],)


@register("GatherV2", "Gather", "ResourceGather")
def _gather(ctx, node, params, indices, *axis):
    if hasattr(params, "read"):
        params = params.read()
    a = _ints(axis[0])[0] if axis else 0
    return (torch.index_select(params, a, indices.reshape(-1).long()).reshape(
        *params.shape[:a], *indices.shape, *params.shape[a + 1:]),)


@register("OneHot")
def _one_hot(ctx, node, idx, depth, on, off):
    d = int(depth.item())
    oh = F.one_hot(idx.long().clamp_min(0), d).to(on.dtype)
    oh = oh * (idx.unsqueeze(-1) >= 0)
    return (oh * on + (1 - oh) * off,)


# ------------------------------------------------------------------ reductions
def _reduce(fn):
    def k(ctx, node, x, axes):
        ax = _ints(axes)
        keep = node.attr("keep_dims", False)
        if not ax:
            return (x,)
        ax = [a % x.dim() for a in ax]
        return (fn(x, ax, keep),)

    return k


register("Mean")(_reduce(lambda x, a, k: x.mean(dim=a, keepdim=k)))
register("Sum")(_reduce(lambda x, a, k: x.sum(dim=a, keepdim=k)))
register("Prod")(_reduce(lambda x, a, k: _multi(torch.prod, x, a, k)))
register("Max")(_reduce(lambda x, a, k: torch.amax(x, dim=a, keepdim=k)))
register("Min")(_reduce(lambda x, a, k: torch.amin(x, dim=a, keepdim=k)))
register("All")(_reduce(lambda x, a, k: _multi(torch.all, x, a, k)))
register("Any")(_reduce(lambda x, a, k: _multi(torch.any, x, a, k)))


def _multi(fn, x, axes, keep):
    for a in sorted(axes, reverse=True):
        x = fn(x, dim=a, keepdim=keep)
    return x


@register("ArgMax")
def _argmax(ctx, node, x, axis):
    return (torch.argmax(x, dim=_ints(axis)[0]).to(node.attr("output_type", DataType.INT64).torch),)


@register("ArgMin")
def _argmin(ctx, node, x, axis):
    return (torch.argmin(x, dim=_ints(axis)[0]).to(node.attr("output_type", DataType.INT64).torch),)


@register("TopKV2", "TopK")
def _topk(ctx, node, x, *k):
    kk = _ints(k[0])[0] if k else node.attr("k")
    v, i = torch.topk(x, kk, dim=-1, largest=True, sorted=node.attr("sorted", True))
    return (v, i.to(torch.int32))


@register("Softmax")
def _softmax(ctx, node, x):
    return (torch.softmax(x.float(), dim=-1).to(x.dtype),)


@register("LogSoftmax")
def _log_softmax(ctx, node, x):
    return (torch.log_softmax(x.float(), dim=-1).to(x.dtype),)


@register("SoftmaxCrossEntropyWithLogits")
def _sxent(ctx, node, logits, labels):
    lsm = torch.log_softmax(logits, -1)
    loss = -(labels * lsm).sum(-1)
    return (loss, torch.softmax(logits, -1) - labels)


@register("SigmoidCrossEntropyWithLogits")
def _sig_xent(ctx, node, labels, logits):
    return (F.binary_cross_entropy_with_logits(logits, labels, reduction="none"),)


@register("RandomUniform")
def _rand_uniform(ctx, node, shape):
    return (torch.rand(tuple(_ints(shape)), dtype=node.attr("dtype").torch, device=ctx.device),)


@register("RandomStandardNormal")
def _rand_normal(ctx, node, shape):
    return (torch.randn(tuple(_ints(shape)), dtype=node.attr("dtype").torch, device=ctx.device),)


@register("TruncatedNormal")
def _trunc_normal(ctx, node, shape):
    t = torch.empty(tuple(_ints(shape)), dtype=node.attr("dtype").torch, device=ctx.device)
    torch.nn.init.trunc_normal_(t, std=1.0, a=-2.0, b=2.0)
    return (t,)


__all__ = ["VarRef", "FailedPreconditionError", "dtype_of"]
