"""Tensor values flowing through graphs.

Numeric tensors are plain ``torch.Tensor`` objects (host or HBM).  TF ``STRING`` tensors
have no torch equivalent; :class:`StringTensor` holds them as a numpy object array of
``bytes`` and converts to/from the TF1 STRING buffer layout (u64 offsets + varint-prefixed
elements), the layout the reference packs by hand in
``LIB/types/TensorInjections.scala:49-78``.
"""
from __future__ import annotations

from typing import Iterable, Sequence

import numpy as np
import torch

from .dtypes import DataType


class StringTensor:
    __slots__ = ("array",)

    def __init__(self, values, shape: Sequence[int] | None = None):
        if isinstance(values, StringTensor):
            arr = values.array
        elif isinstance(values, (bytes, bytearray, str)):
            arr = np.empty((), dtype=object)
            arr[()] = _as_bytes(values)
        else:
            flat = [_as_bytes(v) for v in _flatten(values)]
            arr = np.empty(len(flat), dtype=object)
            arr[:] = flat
            if shape is None:
                shape = np.shape(np.asarray(values, dtype=object)) if not isinstance(values, np.ndarray) else values.shape
        if shape is not None:
            arr = arr.reshape(tuple(shape))
        self.array = arr

    # ------------------------------------------------------------------ properties
    @property
    def shape(self) -> tuple[int, ...]:
        return tuple(self.array.shape)

    @property
    def dtype(self) -> DataType:
        return DataType.STRING

    def dim(self) -> int:
        return self.array.ndim

    def numel(self) -> int:
        return int(self.array.size)

    def __len__(self):
        return len(self.array)

    def __getitem__(self, i):
        v = self.array[i]
        return StringTensor(v) if isinstance(v, np.ndarray) else v

    def item(self) -> bytes:
        if self.array.size != 1:
            raise ValueError("item() on a non-scalar STRING tensor")
        return self.array.reshape(-1)[0]

    def tolist(self):
        return self.array.tolist()

    def reshape(self, *shape) -> "StringTensor":
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        return StringTensor(self.array.reshape(shape))

    # ------------------------------------------------------------------ TF1 buffer
    def to_buffer(self) -> bytes:
        from .. import _ext

        return _ext.native().string_tensor_pack(list(self.array.reshape(-1)))

    @classmethod
    def from_buffer(cls, buf: bytes, shape: Sequence[int]) -> "StringTensor":
        from .. import _ext

        n = int(np.prod(shape)) if len(shape) else 1
        vals = _ext.native().string_tensor_unpack(buf, n)
        return cls(vals, shape)

    def __eq__(self, other):
        if not isinstance(other, StringTensor):
            return NotImplemented
        return self.shape == other.shape and all(a == b for a, b in zip(self.array.reshape(-1), other.array.reshape(-1)))

    def __repr__(self):
        return f"StringTensor(shape={self.shape}, values={self.array.reshape(-1)[:4].tolist()}{'...' if self.numel() > 4 else ''})"


def _as_bytes(v) -> bytes:
    if isinstance(v, bytes):
        return v
    if isinstance(v, (bytearray, memoryview)):
        return bytes(v)
    if isinstance(v, str):
        return v.encode("utf-8")
    if hasattr(v, "SerializeToString"):
        return v.SerializeToString()
    raise TypeError(f"cannot convert {type(v).__name__} to a STRING element")


def _flatten(values) -> Iterable:
    if isinstance(values, np.ndarray):
        yield from values.reshape(-1)
        return
    for v in values:
        if isinstance(v, (list, tuple, np.ndarray)) and not isinstance(v, (bytes, str)):
            yield from _flatten(v)
        else:
            yield v


Tensor = torch.Tensor | StringTensor


def dtype_of(t) -> DataType:
    if isinstance(t, StringTensor):
        return DataType.STRING
    return DataType.from_torch(t.dtype)


def shape_of(t) -> tuple[int, ...]:
    return tuple(t.shape)


def as_tensor(value, dtype: DataType | None = None, device=None):
    """Converts python / numpy values to a graph tensor."""
    if isinstance(value, (StringTensor, torch.Tensor)):
        t = value
    elif isinstance(value, (bytes, bytearray, str)):
        t = StringTensor(value)
    else:
        arr = np.asarray(value)
        if arr.dtype.kind in ("S", "O", "U"):
            t = StringTensor(arr if arr.dtype == object else arr.astype(object))
        else:
            t = torch.from_numpy(np.ascontiguousarray(arr))
    if dtype is not None and not isinstance(t, StringTensor):
        dtype = DataType.of(dtype)
        if dtype == DataType.STRING:
            raise TypeError("numeric value given for a STRING tensor")
        t = t.to(dtype.torch)
    if device is not None and isinstance(t, torch.Tensor):
        t = t.to(device)
    return t
