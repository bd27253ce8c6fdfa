"""``TensorName`` ("op:index") and typed-tensor tagging.

* ``TensorName`` — same grammar as ``LIB/types/TensorName.scala:6-20``: ``"op"`` means
  output 0, ``"op:k"`` output k, more than one colon is an error.
* ``TypedTensor`` / ``Rank`` — the reference tags TF tensors with phantom types
  ``TypedTensor[K <: Product, V]`` (``TFS/package.scala:28-60``, ``TFS/Rank.scala``).
  Python has no phantom types; we keep the vocabulary as runtime-checked tags used when
  a signature binds its inputs and outputs (``tagged_as`` validates rank and dtype).
"""
from __future__ import annotations

from dataclasses import dataclass

from .dtypes import DataType


@dataclass(frozen=True)
class TensorName:
    name: str
    index: int = 0

    @classmethod
    def parse(cls, s: str) -> "TensorName":
        parts = s.split(":")
        if len(parts) == 1:
            return cls(parts[0], 0)
        if len(parts) == 2:
            if not parts[1].lstrip("-").isdigit():
                raise ValueError(f"invalid tensor name {s!r}")
            return cls(parts[0], int(parts[1]))
        raise ValueError(f"invalid tensor name {s!r}")

    def __str__(self):
        return f"{self.name}:{self.index}"

    # reference-style accessor names
    @property
    def op(self) -> str:
        return self.name


class Rank:
    """Rank markers ``Rank.of(k)``; ``Rank0D`` … ``Rank25D`` mirror `` `0D` `` … `` `25D` ``."""

    __slots__ = ("k",)
    _cache: dict[int, "Rank"] = {}

    def __init__(self, k: int):
        self.k = k

    @classmethod
    def of(cls, k: int) -> "Rank":
        if k not in cls._cache:
            cls._cache[k] = Rank(k)
        return cls._cache[k]

    def __repr__(self):
        return f"Rank({self.k}D)"


for _k in range(26):
    globals()[f"Rank{_k}D"] = Rank.of(_k)
ANY_RANK = None


@dataclass(frozen=True)
class TypeTag:
    """``TensorTypeTag[K, V]`` — expected rank (``None`` = any) and element type."""

    rank: int | None
    dtype: DataType | None

    def check(self, t) -> None:
        from .tensor import dtype_of

        if self.rank is not None and t.dim() != self.rank:
            raise TypeError(f"expected a rank-{self.rank} tensor, got shape {tuple(t.shape)}")
        if self.dtype is not None and dtype_of(t) != self.dtype:
            raise TypeError(f"expected {self.dtype.name} tensor, got {dtype_of(t).name}")


def TypedTensor(rank, dtype) -> TypeTag:  # noqa: N802 - mirrors the reference's type name
    r = rank.k if isinstance(rank, Rank) else rank
    return TypeTag(r, DataType.of(dtype) if dtype is not None else None)


def tagged_as(t, tag: TypeTag):
    """``t.taggedAs[T]`` with a runtime check; returns ``t`` unchanged."""
    tag.check(t)
    return t


def tagged_with(t, rank, dtype):
    return tagged_as(t, TypedTensor(rank, dtype))
