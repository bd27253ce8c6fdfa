"""Data types and their TensorFlow wire codes.

The reference maps only FLOAT=1, DOUBLE=2, INT32=3, STRING=7, INT64=9, BOOL=10 and rejects
everything else (``LIB/util/TFUtils.java:10-32``).  We keep those codes bit-exact (they
appear in serialized TensorValues) and add the types the MI355X paths need: UINT8 (raw
images), INT8/INT16, BFLOAT16 (14), HALF (19) and the OCP FP8 formats CDNA4 computes in
(FLOAT8_E5M2=24, FLOAT8_E4M3FN=25; *not* the MI300 ``fnuz`` variants).
"""
from __future__ import annotations

import enum

import numpy as np
import torch


class DataType(enum.IntEnum):
    FLOAT = 1
    DOUBLE = 2
    INT32 = 3
    UINT8 = 4
    INT16 = 5
    INT8 = 6
    STRING = 7
    INT64 = 9
    BOOL = 10
    BFLOAT16 = 14
    UINT16 = 17
    HALF = 19
    RESOURCE = 20
    UINT32 = 22
    UINT64 = 23
    FLOAT8_E5M2 = 24
    FLOAT8_E4M3FN = 25

    # ----------------------------------------------------------------- conversions
    @property
    def torch(self) -> torch.dtype:
        try:
            return _TO_TORCH[self]
        except KeyError:
            raise TypeError(f"{self.name} has no torch dtype") from None

    @property
    def numpy(self):
        try:
            return _TO_NUMPY[self]
        except KeyError:
            raise TypeError(f"{self.name} has no numpy dtype") from None

    @property
    def itemsize(self) -> int:
        if self == DataType.STRING:
            raise TypeError("STRING has no fixed item size")
        return torch.empty((), dtype=self.torch).element_size()

    @property
    def is_floating(self) -> bool:
        return self in (DataType.FLOAT, DataType.DOUBLE, DataType.BFLOAT16, DataType.HALF,
                        DataType.FLOAT8_E5M2, DataType.FLOAT8_E4M3FN)

    @classmethod
    def from_torch(cls, dt: torch.dtype) -> "DataType":
        try:
            return _FROM_TORCH[dt]
        except KeyError:
            raise TypeError(f"unsupported torch dtype {dt}") from None

    @classmethod
    def from_numpy(cls, dt) -> "DataType":
        dt = np.dtype(dt)
        if dt.kind in ("S", "O", "U"):
            return cls.STRING
        try:
            return _FROM_NUMPY[dt]
        except KeyError:
            raise TypeError(f"unsupported numpy dtype {dt}") from None

    @classmethod
    def of(cls, x) -> "DataType":
        if isinstance(x, DataType):
            return x
        if isinstance(x, int):
            return cls(x)
        if isinstance(x, torch.dtype):
            return cls.from_torch(x)
        if isinstance(x, str):
            return cls[x.upper()]
        return cls.from_numpy(x)


_TO_TORCH = {
    DataType.FLOAT: torch.float32,
    DataType.DOUBLE: torch.float64,
    DataType.INT32: torch.int32,
    DataType.UINT8: torch.uint8,
    DataType.INT16: torch.int16,
    DataType.INT8: torch.int8,
    DataType.INT64: torch.int64,
    DataType.BOOL: torch.bool,
    DataType.BFLOAT16: torch.bfloat16,
    DataType.UINT16: torch.uint16,
    DataType.HALF: torch.float16,
    DataType.UINT32: torch.uint32,
    DataType.UINT64: torch.uint64,
    DataType.FLOAT8_E5M2: torch.float8_e5m2,
    DataType.FLOAT8_E4M3FN: torch.float8_e4m3fn,
}
_FROM_TORCH = {v: k for k, v in _TO_TORCH.items()}

_TO_NUMPY = {
    DataType.FLOAT: np.dtype(np.float32),
    DataType.DOUBLE: np.dtype(np.float64),
    DataType.INT32: np.dtype(np.int32),
    DataType.UINT8: np.dtype(np.uint8),
    DataType.INT16: np.dtype(np.int16),
    DataType.INT8: np.dtype(np.int8),
    DataType.INT64: np.dtype(np.int64),
    DataType.BOOL: np.dtype(np.bool_),
    DataType.UINT16: np.dtype(np.uint16),
    DataType.HALF: np.dtype(np.float16),
    DataType.UINT32: np.dtype(np.uint32),
    DataType.UINT64: np.dtype(np.uint64),
    DataType.STRING: np.dtype(object),
}
_FROM_NUMPY = {v: k for k, v in _TO_NUMPY.items() if k != DataType.STRING}

# Codes accepted by the reference's TFUtils (kept for strict-compat mode).
REFERENCE_WIRE_CODES = frozenset({1, 2, 3, 7, 9, 10})


def get_value(dt) -> int:
    """``TFUtils.getValue``: DataType -> wire code."""
    return int(DataType.of(dt))


def get_data_type(code: int, strict: bool = False) -> DataType:
    """``TFUtils.getDataType``: wire code -> DataType (strict = reference's 6 codes only)."""
    if strict and code not in REFERENCE_WIRE_CODES:
        raise ValueError(f"unsupported data type code {code}")
    try:
        return DataType(code)
    except ValueError:
        raise ValueError(f"unsupported data type code {code}") from None
