"""TensorProto ↔ tensor conversion (TF ``tensor_util.make_tensor_proto`` / ``MakeNdarray``)."""
from __future__ import annotations

import numpy as np
import torch

from ..proto.messages import TensorProto, TensorShapeProto
from ..types.dtypes import DataType
from ..types.tensor import StringTensor, as_tensor, dtype_of


def make_tensor_proto(value, dtype=None, shape=None) -> TensorProto:
    t = as_tensor(value, dtype=None)
    dt = DataType.of(dtype) if dtype is not None else dtype_of(t)
    if shape is None:
        shape = tuple(t.shape)
    tp = TensorProto(dtype=int(dt), tensor_shape=TensorShapeProto.of(shape))
    if dt == DataType.STRING:
        if not isinstance(t, StringTensor):
            raise TypeError("STRING proto needs bytes values")
        tp.string_val = list(t.array.reshape(-1))
        return tp
    if isinstance(t, StringTensor):
        raise TypeError("numeric proto given bytes values")
    t = t.detach().to("cpu").to(dt.torch).contiguous()
    if t.numel() != int(np.prod(shape)):
        t = t.expand(tuple(shape)).contiguous()
    tp.tensor_content = t.reshape(-1).view(torch.uint8).numpy().tobytes() if t.numel() else b""
    return tp


def _fill(vals: np.ndarray, n: int) -> np.ndarray:
    if vals.size == n:
        return vals
    if vals.size == 0:
        return np.zeros(n, dtype=vals.dtype)
    out = np.empty(n, dtype=vals.dtype)
    out[: vals.size] = vals
    out[vals.size:] = vals[-1]  # TF repeats the last value
    return out


def tensor_from_proto(tp: TensorProto, device=None):
    dt = DataType(tp.dtype)
    shape = tuple(tp.tensor_shape.as_list() or []) if tp.tensor_shape is not None else ()
    n = int(np.prod(shape)) if shape else 1
    if dt == DataType.STRING:
        vals = list(tp.string_val)
        if len(vals) < n:
            vals = vals + [vals[-1] if vals else b""] * (n - len(vals))
        return StringTensor(vals, shape)
    if tp.tensor_content:
        raw = np.frombuffer(tp.tensor_content, dtype=np.uint8).copy()
        t = torch.from_numpy(raw).view(dt.torch).reshape(shape)
    else:
        if dt in (DataType.FLOAT,):
            vals = np.asarray(tp.float_val, dtype=np.float32)
        elif dt == DataType.DOUBLE:
            vals = np.asarray(tp.double_val, dtype=np.float64)
        elif dt in (DataType.INT32, DataType.INT16, DataType.INT8, DataType.UINT8, DataType.UINT16):
            vals = np.asarray(tp.int_val, dtype=np.int64)
        elif dt == DataType.INT64:
            vals = np.asarray(tp.int64_val, dtype=np.int64)
        elif dt == DataType.BOOL:
            vals = np.asarray(tp.bool_val, dtype=np.bool_)
        elif dt in (DataType.HALF, DataType.BFLOAT16):
            bits = np.asarray(tp.half_val, dtype=np.int64).astype(np.uint16)
            t = torch.from_numpy(_fill(bits, n).astype(np.int16)).view(dt.torch).reshape(shape)
            return t.to(device) if device is not None else t
        elif dt == DataType.UINT32:
            vals = np.asarray(tp.uint32_val, dtype=np.int64)
        elif dt == DataType.UINT64:
            vals = np.asarray(tp.uint64_val, dtype=np.uint64)
        else:
            raise TypeError(f"cannot decode TensorProto of dtype {dt.name}")
        t = torch.from_numpy(_fill(vals, n)).to(dt.torch).reshape(shape)
    return t.to(device) if device is not None else t
