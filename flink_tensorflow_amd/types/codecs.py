"""Conversions between Python values and graph tensors ("injections").

Parity map (reference → here):

* ``TensorInjections`` (``LIB/types/TensorInjections.scala:19-274``):
  scalars ↔ 0-D tensors, arrays ↔ 1-D tensors (inverse squeezes, rank ≤ 1), TensorValue
  ↔ tensor with a rank/dtype check on invert, protobuf message ↔ STRING scalar, list of
  messages ↔ STRING vector.  The list packing is sized dynamically and is invertible
  (the reference caps it at 10,000 bytes and leaves the inverse ``???``, B3).
* ``Arrays`` (``TFS/Arrays.scala:12-61``) → ``array_to_tensor`` / ``tensor_to_array``.
* ``ByteStrings`` (``TFS/ByteStrings.scala:15-39``) → ``bytes_to_tensor`` /
  ``tensor_to_bytes``.
* Flink↔TF bridge (``LIB/package.scala:9-33``) → ``TensorValue.from_tensor`` /
  ``TensorValue.to_tensor`` plus ``to_value``.

``Injection`` objects expose ``apply``/``invert`` for code written against the
reference's bijection style.
"""
from __future__ import annotations

from typing import Callable, Generic, Sequence, TypeVar

import numpy as np
import torch

from .dtypes import DataType
from .names import TypeTag
from .tensor import StringTensor, as_tensor, dtype_of
from .tensor_value import TensorValue

A = TypeVar("A")
B = TypeVar("B")


class Injection(Generic[A, B]):
    def __init__(self, apply: Callable[[A], B], invert: Callable[[B], A]):
        self._apply = apply
        self._invert = invert

    def apply(self, a: A) -> B:
        return self._apply(a)

    def invert(self, b: B) -> A:
        return self._invert(b)

    __call__ = apply

    def and_then(self, other: "Injection") -> "Injection":
        return Injection(lambda a: other.apply(self.apply(a)), lambda c: self.invert(other.invert(c)))


# ------------------------------------------------------------------ scalars / arrays
def scalar_to_tensor(v, dtype=None):
    if isinstance(v, (bytes, str)):
        return StringTensor(v)
    if dtype is None:
        if isinstance(v, bool):
            dtype = DataType.BOOL
        elif isinstance(v, (int, np.integer)):
            dtype = DataType.INT64
        else:
            dtype = DataType.FLOAT
    return torch.tensor(v, dtype=DataType.of(dtype).torch)


def tensor_to_scalar(t):
    if isinstance(t, StringTensor):
        return t.item()
    if t.numel() != 1:
        raise ValueError(f"expected a scalar tensor, got shape {tuple(t.shape)}")
    return t.reshape(()).item()


def array_to_tensor(a, dtype=None) -> torch.Tensor:
    arr = np.asarray(a)
    if arr.ndim != 1:
        raise ValueError("arrays map to rank-1 tensors")
    t = torch.from_numpy(np.ascontiguousarray(arr))
    return t.to(DataType.of(dtype).torch) if dtype is not None else t


def tensor_to_array(t) -> np.ndarray:
    """Inverse of ``array_to_tensor``: squeezes unit dims, then requires rank ≤ 1."""
    if isinstance(t, StringTensor):
        arr = t.array
    else:
        tt = t.detach().cpu()
        arr = (tt.float() if tt.dtype == torch.bfloat16 else tt).numpy()
    arr = np.squeeze(arr)
    if arr.ndim > 1:
        raise ValueError(f"cannot squeeze shape {t.shape} to a vector")
    return arr.reshape(-1)


# ------------------------------------------------------------------ bytes / messages
def bytes_to_tensor(b: bytes) -> StringTensor:
    return StringTensor(bytes(b))


def tensor_to_bytes(t: StringTensor) -> bytes:
    if not isinstance(t, StringTensor) or t.dim() != 0:
        raise TypeError("expected a 0-D STRING tensor")
    return t.item()


def message_to_tensor(msg) -> StringTensor:
    return StringTensor(msg.SerializeToString())


def tensor_to_message(t: StringTensor, cls):
    return cls.FromString(tensor_to_bytes(t))


def messages_to_tensor(msgs: Sequence) -> StringTensor:
    """``List[Message] → STRING[N]`` (dynamic size; no 10,000-byte cap)."""
    return StringTensor([m.SerializeToString() if hasattr(m, "SerializeToString") else bytes(m) for m in msgs],
                        shape=(len(msgs),))


def tensor_to_messages(t: StringTensor, cls) -> list:
    if not isinstance(t, StringTensor):
        raise TypeError("expected a STRING tensor")
    return [cls.FromString(b) for b in t.array.reshape(-1)]


# ------------------------------------------------------------------ TensorValue
def value_to_tensor(v: TensorValue, tag: TypeTag | None = None, device=None):
    t = v.to_tensor(device=device)
    if tag is not None:
        tag.check(t)
    return t


def to_value(t) -> TensorValue:
    """``RichTensor.toValue`` (``LIB/package.scala:24-32``)."""
    return TensorValue.from_tensor(t)


# ------------------------------------------------------------------ injections
class TensorInjections:
    """Named injections mirroring ``TensorInjections``' implicits."""

    @staticmethod
    def bytes2Tensor() -> Injection:
        return Injection(bytes_to_tensor, tensor_to_bytes)

    @staticmethod
    def message2Tensor(cls) -> Injection:
        return Injection(message_to_tensor, lambda t: tensor_to_message(t, cls))

    @staticmethod
    def messages2Tensor(cls) -> Injection:
        return Injection(messages_to_tensor, lambda t: tensor_to_messages(t, cls))

    @staticmethod
    def array2Tensor(dtype) -> Injection:
        return Injection(lambda a: array_to_tensor(a, dtype), tensor_to_array)

    @staticmethod
    def scalar2Tensor(dtype) -> Injection:
        return Injection(lambda v: scalar_to_tensor(v, dtype), tensor_to_scalar)

    @staticmethod
    def tensorValue2Tensor(rank: int | None = None, dtype=None) -> Injection:
        tag = TypeTag(rank, DataType.of(dtype) if dtype is not None else None)

        def inv(t):
            tag.check(t)
            return TensorValue.from_tensor(t)

        return Injection(lambda v: value_to_tensor(v, tag), inv)


def to_graph_tensor(x, device=None):
    """Best-effort conversion used by ``ModelFunction`` when feeding raw python values."""
    if isinstance(x, TensorValue):
        return x.to_tensor(device=device)
    if isinstance(x, list) and x and hasattr(x[0], "SerializeToString"):
        return messages_to_tensor(x)
    if hasattr(x, "SerializeToString"):
        return message_to_tensor(x)
    return as_tensor(x, device=device)


__all__ = [
    "Injection", "TensorInjections", "scalar_to_tensor", "tensor_to_scalar", "array_to_tensor", "tensor_to_array",
    "bytes_to_tensor", "tensor_to_bytes", "message_to_tensor", "tensor_to_message", "messages_to_tensor",
    "tensor_to_messages", "value_to_tensor", "to_value", "to_graph_tensor", "dtype_of",
]
