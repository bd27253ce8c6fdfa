"""TensorBundle V2 checkpoint reader/writer (TF ``SaveV2``/``RestoreV2`` on-disk format).

Layout for a checkpoint ``prefix``::

    prefix.index                    LevelDB table: "" -> BundleHeaderProto,
                                    name -> BundleEntryProto{dtype, shape, shard, offset, size, crc32c}
    prefix.data-00000-of-0000N      concatenated little-endian tensor payloads

STRING tensors are stored TF-style: ``varint64 len[i]… | u32 masked_crc(lengths) | bytes…``.
Their entry checksum is NOT a CRC of that raw payload: like TF's ``WriteStringTensor`` it
covers each length as a fixed-width little-endian integer (u32, or u64 above 4 GiB), then
the 4 stored length-checksum bytes, then the string bytes (``_string_crc``).
The table build/parse and CRC32C run in C++ (``_native.sstable_*``, SSE4.2 ``crc32``).
The reference reaches this format only through the graph's saver subgraph
(``LIB/io/Saver.scala:55-89``); we implement it natively so both the
graph-level saver and the streaming checkpoint backend (§5.4) share it.  Writing from HBM
goes through one device→host copy per tensor.
"""
from __future__ import annotations

import os
import struct
from typing import Iterable, Mapping

import numpy as np
import torch

from .. import _ext
from ..proto.messages import BundleEntryProto, BundleHeaderProto, TensorShapeProto, VersionDef
from ..proto.wire import decode_varint, encode_varint
from ..types.dtypes import DataType
from ..types.tensor import StringTensor, dtype_of


class DataLossError(IOError):
    """Checksum mismatch in a checkpoint (corrupt shard or index)."""


def _mask(crc: int) -> int:
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def data_filename(prefix: str, shard: int, num_shards: int) -> str:
    return f"{prefix}.data-{shard:05d}-of-{num_shards:05d}"


def index_filename(prefix: str) -> str:
    return f"{prefix}.index"


def _fixed_lengths(lens) -> bytes:
    return b"".join(struct.pack("<I", n) if n <= 0xFFFFFFFF else struct.pack("<Q", n) for n in lens)


def _string_crc(lens, cks: bytes, elems) -> int:
    """Unmasked entry CRC of a STRING tensor: fixed-width lengths, the stored length
    checksum, then every element's bytes."""
    nat = _ext.native()
    crc = nat.crc32c(_fixed_lengths(lens))
    crc = nat.crc32c(cks, crc)
    for e in elems:
        crc = nat.crc32c(e, crc)
    return crc


def _tensor_bytes(t) -> tuple[bytes, int]:
    """(payload, masked entry crc32c)."""
    nat = _ext.native()
    if isinstance(t, StringTensor):
        elems = [bytes(e) for e in t.array.reshape(-1)]
        lens = [len(e) for e in elems]
        cks = struct.pack("<I", _mask(nat.crc32c(_fixed_lengths(lens))))
        payload = b"".join(encode_varint(n) for n in lens) + cks + b"".join(elems)
        return payload, _mask(_string_crc(lens, cks, elems))
    t = t.detach().to("cpu").contiguous()
    payload = t.reshape(-1).view(torch.uint8).numpy().tobytes() if t.numel() else b""
    return payload, _mask(nat.crc32c(payload))


class BundleWriter:
    """Writes one shard (``shard_id`` of ``num_shards``) plus, for a single shard, the index."""

    def __init__(self, prefix: str, shard_id: int = 0, num_shards: int = 1):
        self.prefix = prefix
        self.shard_id = shard_id
        self.num_shards = num_shards
        self.entries: dict[str, BundleEntryProto] = {}
        d = os.path.dirname(prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        self._path = data_filename(prefix, shard_id, num_shards)
        self._f = open(self._path + ".tmp", "wb")
        self._off = 0

    def add(self, name: str, tensor) -> None:
        if name in self.entries:
            raise ValueError(f"duplicate tensor {name!r} in bundle")
        payload, crc = _tensor_bytes(tensor)
        e = BundleEntryProto(dtype=int(dtype_of(tensor)), shape=TensorShapeProto.of(tensor.shape),
                             shard_id=self.shard_id, offset=self._off, size=len(payload), crc32c=crc)
        self._f.write(payload)
        self._off += len(payload)
        self.entries[name] = e

    def finish(self, write_index: bool = True) -> dict[str, BundleEntryProto]:
        self._f.close()
        os.replace(self._path + ".tmp", self._path)
        if write_index:
            write_index_file(self.prefix, self.entries, self.num_shards)
        return self.entries


def write_index_file(prefix: str, entries: Mapping[str, BundleEntryProto], num_shards: int) -> None:
    header = BundleHeaderProto(num_shards=num_shards, version=VersionDef(producer=1))
    items = [(b"", header.encode())] + [(k.encode(), entries[k].encode()) for k in sorted(entries)]
    data = _ext.native().sstable_build(items)
    tmp = index_filename(prefix) + ".tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, index_filename(prefix))


def save_tensors(prefix: str, tensors: Mapping[str, object]) -> None:
    w = BundleWriter(prefix)
    for k in sorted(tensors):
        w.add(k, tensors[k])
    w.finish()


class BundleReader:
    def __init__(self, prefix: str, verify: bool = True):
        self.prefix = prefix
        self.verify = verify
        path = index_filename(prefix)
        if not os.path.exists(path):
            raise FileNotFoundError(f"checkpoint index not found: {path}")
        with open(path, "rb") as f:
            raw = f.read()
        try:
            items = _ext.native().sstable_parse(raw, verify)
        except RuntimeError as e:
            raise DataLossError(str(e)) from None
        self.header = BundleHeaderProto()
        self.entries: dict[str, BundleEntryProto] = {}
        for k, v in items:
            if k == b"":
                self.header = BundleHeaderProto.decode(v)
            else:
                self.entries[k.decode()] = BundleEntryProto.decode(v)
        if self.header.endianness != BundleHeaderProto.LITTLE:
            raise NotImplementedError("big-endian bundles are not supported")
        self._files: dict[int, object] = {}

    def keys(self) -> list[str]:
        return sorted(self.entries)

    def __contains__(self, name):
        return name in self.entries

    def _file(self, shard: int):
        f = self._files.get(shard)
        if f is None:
            f = open(data_filename(self.prefix, shard, max(1, self.header.num_shards)), "rb")
            self._files[shard] = f
        return f

    def dtype_and_shape(self, name: str):
        e = self.entries[name]
        return DataType(e.dtype), tuple(e.shape.as_list() or [])

    def read(self, name: str, device=None):
        if name not in self.entries:
            raise KeyError(f"tensor {name!r} not found in checkpoint {self.prefix}")
        e = self.entries[name]
        f = self._file(e.shard_id)
        f.seek(e.offset)
        payload = f.read(e.size)
        if len(payload) != e.size:
            raise DataLossError(f"truncated data for {name!r}")
        dt = DataType(e.dtype)
        shape = tuple(e.shape.as_list() or [])
        if dt == DataType.STRING:
            n = int(np.prod(shape)) if shape else 1
            off = 0
            lens = []
            for _ in range(n):
                ln, off = decode_varint(payload, off)
                lens.append(ln)
            cks = payload[off:off + 4]
            off += 4
            vals = []
            for ln in lens:
                vals.append(payload[off:off + ln])
                off += ln
            if self.verify:
                if struct.unpack("<I", cks)[0] != _mask(_ext.native().crc32c(_fixed_lengths(lens))):
                    raise DataLossError(f"length checksum mismatch for string tensor {name!r} in {self.prefix}")
                if _mask(_string_crc(lens, cks, vals)) != e.crc32c:
                    raise DataLossError(f"checksum mismatch for tensor {name!r} in {self.prefix}")
            return StringTensor(vals, shape)
        if self.verify and _mask(_ext.native().crc32c(payload)) != e.crc32c:
            raise DataLossError(f"checksum mismatch for tensor {name!r} in {self.prefix}")
        t = torch.from_numpy(np.frombuffer(payload, dtype=np.uint8).copy()).view(dt.torch).reshape(shape)
        return t.to(device) if device is not None else t

    def read_all(self, device=None) -> dict[str, object]:
        return {k: self.read(k, device) for k in self.keys()}

    def close(self):
        for f in self._files.values():
            f.close()
        self._files.clear()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def merge_bundles(src_prefixes: Iterable[str], dst_prefix: str, delete_old_dirs: bool = True) -> None:
    """``MergeV2Checkpoints``: renames shard data files under ``dst_prefix`` and writes one index."""
    srcs = list(src_prefixes)
    merged: dict[str, BundleEntryProto] = {}
    n = len(srcs)
    for shard, src in enumerate(srcs):
        r = BundleReader(src, verify=False)
        src_shards = max(1, r.header.num_shards)
        if src_shards != 1:
            raise NotImplementedError("merging multi-shard sources")
        r.close()
        d = os.path.dirname(dst_prefix)
        if d:
            os.makedirs(d, exist_ok=True)
        os.replace(data_filename(src, 0, 1), data_filename(dst_prefix, shard, n))
        for k, e in r.entries.items():
            if k in merged:
                raise ValueError(f"duplicate tensor {k!r} across shards")
            e.shard_id = shard
            merged[k] = e
        os.remove(index_filename(src))
        if delete_old_dirs:
            try:
                os.rmdir(os.path.dirname(src))
            except OSError:
                pass
    write_index_file(dst_prefix, merged, n)
