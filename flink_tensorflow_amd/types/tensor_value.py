"""``TensorValue``: a serializable tensor record for streams.

Parity with ``LIB/types/TensorValue.java:47-264``: a dtype + shape + payload value that
crosses operator boundaries in a fixed binary framing (big-endian header, native-order
payload; ``:141-187``)::

    u8 version=0x01 | i32 dtype | i32 rank | i64 dim[rank] | i32 nbytes | payload

Differences by design:

* the payload may live in host memory (numpy/bytes) **or HBM** (a ``torch.Tensor`` on
  ``cuda``); ``to_tensor(device=...)`` moves it without an extra host copy when the
  payload is already pinned;
* verbatim record copy is correct (the reference's ``copyInternal`` copies ``rank``
  bytes of an ``8*rank``-byte shape — SURVEY §2.10 B1);
* records are picklable through the framing (the reference forbids Java
  serialization, B10), so they can be captured in closures and sent between worker
  processes;
* ``TensorValueBuilder`` sizes LONG payloads with 8 bytes/element (B2).

The codec itself runs in C++ (``_native.tv_*``).
"""
from __future__ import annotations

import io
from typing import BinaryIO, Sequence

import numpy as np
import torch

from .. import _ext
from .dtypes import DataType, get_data_type
from .tensor import StringTensor, as_tensor

VERSION_1 = 0x01


class VersionMismatchException(IOError):
    pass


class TensorValue:
    __slots__ = ("dtype", "_shape", "_payload")

    def __init__(self, dtype=DataType.FLOAT, shape: Sequence[int] = (), payload=None):
        self.dtype = DataType.of(dtype)
        self._shape = tuple(int(d) for d in shape)
        # payload: bytes-like (native order) | numpy array | torch.Tensor (any device)
        self._payload = payload if payload is not None else b""

    # ------------------------------------------------------------------ accessors
    def shape(self) -> tuple[int, ...]:
        """A copy of the shape (reference ``shape()`` copies the tuple, ``:122-124``)."""
        return tuple(self._shape)

    @property
    def rank(self) -> int:
        return len(self._shape)

    @property
    def nbytes(self) -> int:
        p = self._payload
        if isinstance(p, torch.Tensor):
            return p.numel() * p.element_size()
        if isinstance(p, np.ndarray):
            return p.nbytes
        return len(p)

    def binary_length(self) -> int:
        """Framed size: 1 + 4 + 4 + 8*rank + 4 + nbytes (reference ``getBinaryLength``)."""
        return 13 + 8 * self.rank + self.nbytes

    @property
    def device(self):
        p = self._payload
        return p.device if isinstance(p, torch.Tensor) else torch.device("cpu")

    def payload_bytes(self) -> bytes:
        p = self._payload
        if isinstance(p, torch.Tensor):
            p = p.detach().contiguous().cpu()
            if p.dtype in (torch.bfloat16, torch.float8_e4m3fn, torch.float8_e5m2, torch.uint16, torch.uint32,
                           torch.uint64):
                return p.reshape(-1).view(torch.uint8).numpy().tobytes()
            return p.numpy().tobytes()
        if isinstance(p, np.ndarray):
            return np.ascontiguousarray(p).tobytes()
        return bytes(p)

    # ------------------------------------------------------------------ conversions
    @classmethod
    def from_tensor(cls, t, copy: bool = True) -> "TensorValue":
        """``TensorValue.fromTensor`` (``:257-263``); keeps HBM tensors on device."""
        if isinstance(t, StringTensor):
            return cls(DataType.STRING, t.shape, t.to_buffer())
        if not isinstance(t, torch.Tensor):
            t = as_tensor(t)
            if isinstance(t, StringTensor):
                return cls.from_tensor(t)
        t = t.detach()
        if copy:
            t = t.clone() if t.is_cuda else t.contiguous().clone()
        return cls(DataType.from_torch(t.dtype), t.shape, t.contiguous())

    def to_tensor(self, device=None):
        """``TensorValue.toTensor`` (``:131-133``)."""
        if self.dtype == DataType.STRING:
            return StringTensor.from_buffer(self.payload_bytes(), self._shape)
        p = self._payload
        if isinstance(p, torch.Tensor):
            t = p.reshape(self._shape)
        else:
            raw = p if isinstance(p, np.ndarray) else np.frombuffer(bytes(p), dtype=np.uint8)
            raw = np.ascontiguousarray(raw).view(np.uint8)
            if raw.size == 0:
                t = torch.empty(self._shape, dtype=self.dtype.torch)
            else:
                t = torch.from_numpy(raw.copy()).view(self.dtype.torch).reshape(self._shape)
        if device is not None:
            t = t.to(device, non_blocking=True)
        return t

    def to_numpy(self) -> np.ndarray:
        t = self.to_tensor()
        if isinstance(t, StringTensor):
            return t.array
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()

    # ------------------------------------------------------------------ framing
    def to_bytes(self) -> bytes:
        return _ext.native().tv_encode(int(self.dtype), list(self._shape), self.payload_bytes())

    @classmethod
    def from_bytes(cls, data, offset: int = 0, strict: bool = False) -> "TensorValue":
        v, _ = cls.read_from(data, offset, strict)
        return v

    @classmethod
    def read_from(cls, data, offset: int = 0, strict: bool = False) -> tuple["TensorValue", int]:
        try:
            code, shape, payload, nxt = _ext.native().tv_decode(data, offset)
        except RuntimeError as e:
            if "VersionMismatch" in str(e):
                raise VersionMismatchException(str(e)) from None
            raise
        return cls(get_data_type(code, strict), shape, payload), nxt

    def write(self, out: BinaryIO) -> None:
        """``TensorValue.write(DataOutputView)``."""
        out.write(self.to_bytes())

    @classmethod
    def read(cls, inp: BinaryIO, strict: bool = False) -> "TensorValue":
        """``TensorValue.read(DataInputView)`` — reads exactly one framed record."""
        head = inp.read(9)
        if len(head) < 9:
            raise EOFError("end of stream")
        if head[0] != VERSION_1:
            raise VersionMismatchException("incompatible tensor value")
        rank = int.from_bytes(head[5:9], "big")
        rest = inp.read(8 * rank + 4)
        nbytes = int.from_bytes(rest[-4:], "big")
        payload = inp.read(nbytes)
        if len(payload) != nbytes:
            raise EOFError("truncated tensor value payload")
        return cls.from_bytes(head + rest + payload, strict=strict)

    @staticmethod
    def copy_record(data, offset: int = 0) -> tuple[bytes, int]:
        """Verbatim copy of one framed record (fixed ``copyInternal``)."""
        return _ext.native().tv_copy(data, offset)

    @staticmethod
    def encode_many(values: Sequence["TensorValue"]) -> bytes:
        return _ext.native().tv_encode_many([(int(v.dtype), list(v._shape), v.payload_bytes()) for v in values])

    @staticmethod
    def decode_many(data) -> list["TensorValue"]:
        return [TensorValue(c, s, p) for c, s, p in _ext.native().tv_decode_many(data)]

    # ------------------------------------------------------------------ copies
    def copy(self) -> "TensorValue":
        """Shallow copy sharing the payload (reference ``copyTo`` ``:213-217``)."""
        return TensorValue(self.dtype, self._shape, self._payload)

    def deep_copy(self) -> "TensorValue":
        p = self._payload
        if isinstance(p, torch.Tensor):
            p = p.clone()
        elif isinstance(p, np.ndarray):
            p = p.copy()
        else:
            p = bytes(p)
        return TensorValue(self.dtype, self._shape, p)

    def __reduce__(self):
        return (TensorValue.from_bytes, (self.to_bytes(),))

    def __eq__(self, other):
        if not isinstance(other, TensorValue):
            return NotImplemented
        return self.dtype == other.dtype and self._shape == other._shape and self.payload_bytes() == other.payload_bytes()

    def __repr__(self):
        return f"TensorValue(dtype={self.dtype.name}, shape={self._shape}, device={self.device})"

    @staticmethod
    def builder() -> "TensorValueBuilder":
        return TensorValueBuilder()


class TensorValueBuilder:
    """Fluent builder (``LIB/types/TensorValueBuilder.java:13-106``), LONG sized at 8 B."""

    def __init__(self):
        self._dtype: DataType | None = None
        self._shape: tuple[int, ...] | None = None
        self._data = None

    def data_type(self, dt) -> "TensorValueBuilder":
        self._dtype = DataType.of(dt)
        return self

    def shape(self, *dims) -> "TensorValueBuilder":
        if len(dims) == 1 and isinstance(dims[0], (tuple, list)):
            dims = tuple(dims[0])
        self._shape = tuple(int(d) for d in dims)
        return self

    def data(self, values) -> "TensorValueBuilder":
        self._data = values
        return self

    def build(self) -> TensorValue:
        if self._data is None:
            raise ValueError("data not set")
        if isinstance(self._data, (bytes, bytearray, memoryview)):
            if self._dtype is None or self._shape is None:
                raise ValueError("raw buffers need an explicit dtype and shape")
            return TensorValue(self._dtype, self._shape, bytes(self._data))
        arr = np.asarray(self._data)
        dt = self._dtype or DataType.from_numpy(arr.dtype)
        arr = np.ascontiguousarray(arr.astype(dt.numpy, copy=False))
        shape = self._shape if self._shape is not None else arr.shape
        if int(np.prod(shape)) != arr.size:
            raise ValueError(f"shape {shape} does not match {arr.size} elements")
        return TensorValue(dt, shape, arr.tobytes())


def tensor_values_to_stream(values: Sequence[TensorValue]) -> bytes:
    buf = io.BytesIO()
    for v in values:
        v.write(buf)
    return buf.getvalue()
