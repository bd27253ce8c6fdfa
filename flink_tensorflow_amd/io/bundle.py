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
from ..proto.messages import (BundleEntryProto, BundleHeaderProto, TensorShapeProto, TensorSliceExtent, TensorSliceProto,
                               VersionDef)
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

    def add_slice(self, name: str, full_shape, slices, tensor) -> None:
        """Saves ``tensor`` as the slice ``slices`` ([(start, length or -1)] per dim) of
        variable ``name`` of shape ``full_shape`` (a partitioned variable, TF's
        ``BundleWriter::AddSlice``): the full-tensor entry records the shape and the slice
        list, the data goes under the slice's ordered-code key."""
        full_shape = [int(d) for d in full_shape]
        if len(slices) != len(full_shape):
            raise ValueError(f"slice rank {len(slices)} != shape rank {len(full_shape)} for {name!r}")
        want = tuple(full_shape[d] if ln < 0 else ln for d, (_, ln) in enumerate(slices))
        if tuple(tensor.shape) != want:
            raise ValueError(f"slice of {name!r} has shape {tuple(tensor.shape)}, spec wants {want}")
        e = self.entries.get(name)
        if e is None:
            e = BundleEntryProto(dtype=int(dtype_of(tensor)), shape=TensorShapeProto.of(full_shape))
            self.entries[name] = e
        elif [int(d) for d in (e.shape.as_list() or [])] != full_shape or e.dtype != int(dtype_of(tensor)):
            raise ValueError(f"slices of {name!r} disagree on shape / dtype")
        e.slices.append(TensorSliceProto(extent=[TensorSliceExtent(start=st, length=max(0, ln))
                                                 for st, ln in slices]))
        self.add(encode_tensor_name_slice(name, slices), tensor)

    def finish(self, write_index: bool = True) -> dict[str, BundleEntryProto]:
        self._f.close()
        os.replace(self._path + ".tmp", self._path)
        if write_index:
            write_index_file(self.prefix, self.entries, self.num_shards)
        return self.entries


def _kb(key: str) -> bytes:
    """Index keys are byte strings (slice keys are binary OrderedCode); they live in Python
    as str through the surrogateescape round trip."""
    return key.encode("utf-8", "surrogateescape")


def write_index_file(prefix: str, entries: Mapping[str, BundleEntryProto], num_shards: int) -> None:
    header = BundleHeaderProto(num_shards=num_shards, version=VersionDef(producer=1))
    items = [(b"", header.encode())] + [(_kb(k), entries[k].encode()) for k in sorted(entries, key=_kb)]
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


class _PinnedStager:
    """Two reused pinned host buffers for checkpoint reads into HBM: a buffer is refilled
    only after the device copy that last read it has completed (event per buffer)."""

    def __init__(self, chunk: int = 32 << 20):
        self.chunk = chunk
        self.bufs = [torch.empty(chunk, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
        self.events = [None, None]
        self.i = 0

    def acquire(self, device):
        ev = self.events[self.i]
        if ev is not None:
            ev.synchronize()
        return self.bufs[self.i]

    def release(self, device):
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        self.events[self.i] = ev
        self.i ^= 1

    def drain(self):
        for ev in self.events:
            if ev is not None:
                ev.synchronize()
        self.events = [None, None]


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
                self.entries[k.decode("utf-8", "surrogateescape")] = BundleEntryProto.decode(v)
        if self.header.endianness != BundleHeaderProto.LITTLE:
            raise NotImplementedError("big-endian bundles are not supported")
        self._files: dict[int, object] = {}
        self._stager: _PinnedStager | None = None

    def keys(self) -> list[str]:
        """Tensor names (the binary keys of stored slices are not listed)."""
        return sorted(k for k in self.entries if not k.startswith("\x00"))

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
        if e.slices:  # a partitioned variable: assemble the whole tensor from its slices
            return self.read_slice(name, [(0, -1)] * len(e.shape.as_list() or []), device)
        dt = DataType(e.dtype)
        shape = tuple(e.shape.as_list() or [])
        if dt != DataType.STRING and device is not None and torch.device(device).type == "cuda":
            return self._read_to_device(name, e, dt, shape, torch.device(device))
        f = self._file(e.shard_id)
        f.seek(e.offset)
        payload = f.read(e.size)
        if len(payload) != e.size:
            raise DataLossError(f"truncated data for {name!r}")
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

    def _read_to_device(self, name: str, e, dt, shape, device):
        """Payload -> HBM through a reused pinned staging ring: the file is
        read straight into pinned memory (no pageable bounce), checksummed there, and DMA'd
        to the device asynchronously while the next chunk is read."""
        if self._stager is None:
            self._stager = _PinnedStager()
        out = torch.empty(shape, dtype=dt.torch, device=device)
        if e.size != out.numel() * out.element_size():
            # the CRC covers only the stored bytes: a short entry would leave the tail of the
            # device tensor uninitialised (the host path fails the same input in reshape)
            raise DataLossError(f"tensor {name!r} in {self.prefix}: entry holds {e.size} bytes, "
                                f"shape {list(shape)} of {dt.name} needs {out.numel() * out.element_size()}")
        if e.size == 0:
            return out
        dst = out.view(-1).view(torch.uint8) if out.numel() else out
        f = self._file(e.shard_id)
        f.seek(e.offset)
        crc, off = 0, 0
        nat = _ext.native()
        while off < e.size:
            n = min(e.size - off, self._stager.chunk)
            buf = self._stager.acquire(device)
            view = buf.numpy()[:n]
            if f.readinto(memoryview(view)) != n:
                raise DataLossError(f"truncated data for {name!r}")
            if self.verify:
                crc = nat.crc32c(view, crc)
            dst[off:off + n].copy_(buf[:n], non_blocking=True)
            self._stager.release(device)
            off += n
        if self.verify and _mask(crc) != e.crc32c:
            raise DataLossError(f"checksum mismatch for tensor {name!r} in {self.prefix}")
        return out

    def read_slice(self, name: str, slices, device=None):
        """The slice ``slices`` ([(start, length or -1)] per dim) of tensor ``name``: cut from
        a whole stored tensor, or assembled from the stored slices of a partitioned one."""
        if name not in self.entries:
            raise KeyError(f"tensor {name!r} not found in checkpoint {self.prefix}")
        e = self.entries[name]
        full = [int(d) for d in (e.shape.as_list() or [])]
        if len(slices) != len(full):
            raise ValueError(f"slice rank {len(slices)} != rank {len(full)} of {name!r}")
        want = [(st, full[d] - st if ln < 0 else ln) for d, (st, ln) in enumerate(slices)]
        if not e.slices:
            t = self.read(name)
            return t[tuple(slice(st, st + ln) for st, ln in want)].clone().to(device or "cpu")
        out = torch.empty([ln for _, ln in want], dtype=DataType(e.dtype).torch)
        covered = 0
        for sp in e.slices:
            have = [(x.start, full[d] - x.start if x.length <= 0 else x.length) for d, x in enumerate(sp.extent)]
            lo = [max(a, b) for (a, _), (b, _) in zip(want, have)]
            hi = [min(a + la, b + lb) for (a, la), (b, lb) in zip(want, have)]
            if any(h <= l for l, h in zip(lo, hi)):
                continue
            stored = self.read(encode_tensor_name_slice(name, [(x.start, x.length if x.length > 0 else -1)
                                                                for x in sp.extent]))
            src = tuple(slice(l - b, h - b) for l, h, (b, _) in zip(lo, hi, have))
            dst = tuple(slice(l - a, h - a) for l, h, (a, _) in zip(lo, hi, want))
            out[dst] = stored[src]
            covered += int(np.prod([h - l for l, h in zip(lo, hi)]))
        if covered != out.numel():
            raise DataLossError(f"stored slices of {name!r} do not cover the requested slice {slices}")
        return out.to(device) if device is not None else out

    def read_all(self, device=None) -> dict[str, object]:
        return {k: self.read(k, device) for k in self.keys()}

    def close(self):
        for f in self._files.values():
            f.close()
        self._files.clear()
        if self._stager is not None:
            self._stager.drain()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def merge_bundles(src_prefixes: Iterable[str], dst_prefix: str, delete_old_dirs: bool = True) -> None:
    """``MergeV2Checkpoints``: every data shard of every source (sources may themselves be
    multi-shard bundles) is renamed under ``dst_prefix`` with a new shard number, and one
    index is written with the entries' shard ids remapped (data bytes are never copied)."""
    srcs = list(src_prefixes)
    readers = []
    for src in srcs:
        r = BundleReader(src, verify=False)
        r.close()
        readers.append(r)
    total = sum(max(1, r.header.num_shards) for r in readers)
    merged: dict[str, BundleEntryProto] = {}
    d = os.path.dirname(dst_prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    base = 0
    for src, r in zip(srcs, readers):
        n = max(1, r.header.num_shards)
        for sh in range(n):
            os.replace(data_filename(src, sh, n), data_filename(dst_prefix, base + sh, total))
        for k, e in r.entries.items():
            if k in merged and not (e.slices and merged[k].slices):
                raise ValueError(f"duplicate tensor {k!r} across shards")
            if k in merged:  # a partitioned variable saved by several shards: union of its slices
                m = merged[k]
                if (m.dtype != e.dtype or list(m.shape.as_list() or []) != list(e.shape.as_list() or [])):
                    # MergeV2Checkpoints rejects slices of one variable that disagree
                    raise ValueError(f"partitioned tensor {k!r}: shards disagree on its full shape / dtype "
                                     f"({m.shape.as_list()}/{m.dtype} vs {e.shape.as_list()}/{e.dtype})")
                m.slices.extend(e.slices)
                continue
            if not e.slices:
                e.shard_id = base + e.shard_id
            merged[k] = e
        base += n
        os.remove(index_filename(src))
        if delete_old_dirs:
            try:
                os.rmdir(os.path.dirname(src))
            except OSError:
                pass
    write_index_file(dst_prefix, merged, total)


# ------------------------------------------------------------------ partitioned variables
def parse_shape_and_slice(spec: str):
    """``"10 20 0,5:-"`` (SaveV2 / RestoreV2 ``shape_and_slices``) -> (full shape,
    [(start, length or -1)] per dim); ``""`` -> None (the whole tensor)."""
    spec = spec.strip()
    if not spec:
        return None
    parts = spec.split(" ")
    shape, sl = [int(v) for v in parts[:-1]], parts[-1]
    dims = sl.split(":")
    if len(dims) != len(shape):
        raise ValueError(f"slice {sl!r} does not match shape {shape}")
    out = []
    for d in dims:
        if d == "-":
            out.append((0, -1))
        else:
            st, ln = d.split(",")
            out.append((int(st), int(ln)))
    return shape, out


def _ordered_num_increasing(v: int) -> bytes:
    """OrderedCode::WriteNumIncreasing: length byte + big-endian bytes, leading zeros dropped."""
    b = v.to_bytes((v.bit_length() + 7) // 8, "big") if v else b""
    return bytes([len(b)]) + b


def _ordered_string(s: bytes) -> bytes:
    """OrderedCode::WriteString: 0x00 -> 00 ff, 0xff -> ff 00, terminated by 00 01."""
    return _escape(s) + b"\x00\x01"


def _escape(s: bytes) -> bytes:
    out = bytearray()
    for c in s:
        if c == 0:
            out += b"\x00\xff"
        elif c == 0xFF:
            out += b"\xff\x00"
        else:
            out.append(c)
    return bytes(out)


_BITS_TO_LEN = [1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5,
                5, 6, 6, 6, 6, 6, 6, 6, 7, 7, 7, 7, 7, 7, 7, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 10]
_HDR_BITS = [(0, 0), (0x80, 0), (0xC0, 0), (0xE0, 0), (0xF0, 0), (0xF8, 0), (0xFC, 0), (0xFE, 0), (0xFF, 0),
             (0xFF, 0x80), (0xFF, 0xC0)]


def _ordered_signed_increasing(v: int) -> bytes:
    """OrderedCode::WriteSignedNumIncreasing (1-10 bytes, order-preserving for int64)."""
    x = ~v if v < 0 else v
    if x < 64:
        return bytes([(0x80 ^ v) & 0xFF])
    n = _BITS_TO_LEN[x.bit_length()]  # kBitsToLength[Log2Floor64(x) + 1]
    buf = bytearray(((v + (1 << 80)) % (1 << 80)).to_bytes(10, "big"))  # sign-extended to 10 bytes
    b = buf[10 - n:]
    b[0] ^= _HDR_BITS[n][0]
    b[1] ^= _HDR_BITS[n][1]
    return bytes(b)


def encode_tensor_name_slice(name: str, slices) -> str:
    """``checkpoint::EncodeTensorNameSlice``: the index key of one stored slice of a
    partitioned variable (ordered code of 0, the name, the rank, then (start, length) per
    dim with -1 for a full extent).  Written from the TF source's description; no TF is
    available here to pin it byte-for-byte (parity unpinned, round-trip tested)."""
    out = _ordered_num_increasing(0) + _ordered_string(name.encode()) + _ordered_num_increasing(len(slices))
    for st, ln in slices:
        out += _ordered_signed_increasing(int(st)) + _ordered_signed_increasing(int(ln))
    return out.decode("utf-8", "surrogateescape")
