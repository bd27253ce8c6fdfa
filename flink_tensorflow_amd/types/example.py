"""tf.Example construction and batched parsing.

* ``example(("x", feature(1.0)), ...)`` / ``feature(*floats)`` mirror
  ``LIB/util/ExampleBuilder.scala:10-28`` (also duplicated in the reference's
  ``TST/.../util/TestData.scala:22-34``).
* ``parse_example_dense`` is the dense path of TF's ``ParseExample`` op, executed by the
  multithreaded C++ parser in ``_native.parse_examples``.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

from .. import _ext
from ..proto.messages import BytesList, Example, Feature, Features, FloatList, Int64List

FLOAT, INT64, BYTES = 0, 1, 2


def feature(*values: float) -> Feature:
    return Feature(float_list=FloatList(value=[float(v) for v in values]))


def float_feature(values: Sequence[float]) -> Feature:
    return Feature(float_list=FloatList(value=[float(v) for v in values]))


def int64_feature(values: Sequence[int]) -> Feature:
    return Feature(int64_list=Int64List(value=[int(v) for v in values]))


def bytes_feature(values: Sequence[bytes]) -> Feature:
    return Feature(bytes_list=BytesList(value=[bytes(v) for v in values]))


def example(*pairs: tuple[str, Feature], **kw: Feature) -> Example:
    feats = dict(pairs)
    feats.update(kw)
    return Example(features=Features(feature=feats))


def make_example(**features) -> Example:
    """``make_example(x=[1.0], ids=[3, 4])`` — infers the list type from the values."""
    out = {}
    for k, v in features.items():
        if isinstance(v, Feature):
            out[k] = v
            continue
        vals = list(v) if isinstance(v, (list, tuple, np.ndarray)) else [v]
        if vals and isinstance(vals[0], (bytes, str)):
            out[k] = bytes_feature([x.encode() if isinstance(x, str) else x for x in vals])
        elif vals and all(isinstance(x, (int, np.integer)) and not isinstance(x, bool) for x in vals):
            out[k] = int64_feature(vals)
        else:
            out[k] = float_feature(vals)
    return Example(features=Features(feature=out))


def parse_example_dense(serialized: Sequence[bytes], specs: Sequence[tuple[str, int, int, object]],
                        nthreads: int = 8) -> list[np.ndarray]:
    """Parses N serialized Examples.

    ``specs``: ``(key, kind, numel, default)``; kind FLOAT/INT64/BYTES; default ``None`` =
    required.  Returns one ``[N, numel]`` array per spec.
    """
    numeric = [(i, s) for i, s in enumerate(specs) if s[1] != BYTES]
    out: list = [None] * len(specs)
    if numeric:
        nat = [(k, kind, int(n), None if d is None else [float(x) for x in np.asarray(d).reshape(-1)])
               for _, (k, kind, n, d) in numeric]
        arrs = _ext.native().parse_examples([bytes(s) for s in serialized], nat, nthreads)
        for (i, _), a in zip(numeric, arrs):
            out[i] = a
    for i, (k, kind, n, d) in enumerate(specs):
        if kind != BYTES:
            continue
        col = np.empty((len(serialized), n), dtype=object)
        for r, s in enumerate(serialized):
            ex = Example.decode(s)
            f = ex.features.feature.get(k) if ex.features else None
            if f is None or f.bytes_list is None:
                if d is None:
                    raise ValueError(f"Example {r} is missing required feature '{k}'")
                col[r, :] = np.asarray(d, dtype=object).reshape(-1)[:n]
            else:
                if len(f.bytes_list.value) != n:
                    raise ValueError(f"Key: {k}: expected {n} values, got {len(f.bytes_list.value)}")
                col[r, :] = f.bytes_list.value
        out[i] = col
    return out


def parse_example_varlen(serialized: Sequence[bytes], specs: Sequence[tuple[str, int]]):
    """Var-length (``VarLenFeature`` / sparse) features of N serialized Examples as TF's
    sparse triples ``(indices int64 [nnz, 2], values [nnz], dense_shape int64 [2])`` per
    spec ``(key, kind)``; numeric kinds are decoded by the C++ parser, BYTES in Python."""
    ser = [bytes(s) for s in serialized]
    n = len(ser)
    numeric = [(i, (k, kind)) for i, (k, kind) in enumerate(specs) if kind != BYTES]
    csr: list = [None] * len(specs)
    if numeric:
        for (i, _), got in zip(numeric, _ext.native().parse_examples_varlen(ser, [s for _, s in numeric])):
            csr[i] = got
    for i, (k, kind) in enumerate(specs):
        if kind != BYTES:
            continue
        vals, splits = [], [0]
        for s in ser:
            ex = Example.decode(s)
            f = ex.features.feature.get(k) if ex.features else None
            v = list(f.bytes_list.value) if f is not None and f.bytes_list is not None else []
            vals.extend(v)
            splits.append(splits[-1] + len(v))
        csr[i] = (np.asarray(splits, np.int64), np.asarray(vals, dtype=object))
    out = []
    for splits, vals in csr:
        lens = np.diff(splits)
        rows = np.repeat(np.arange(n, dtype=np.int64), lens)
        cols = np.arange(len(vals), dtype=np.int64) - np.repeat(splits[:-1], lens)
        out.append((np.stack([rows, cols], 1) if len(vals) else np.zeros((0, 2), np.int64), vals,
                    np.asarray([n, int(lens.max()) if n else 0], np.int64)))
    return out


def encode_float_examples(columns: dict[str, np.ndarray]) -> list[bytes]:
    """Serializes N examples with float features in C++ (synthetic load generation)."""
    keys = list(columns)
    arrs = [np.ascontiguousarray(np.asarray(columns[k], dtype=np.float32).reshape(len(columns[k]), -1)) for k in keys]
    return _ext.native().encode_float_examples(keys, arrs)
