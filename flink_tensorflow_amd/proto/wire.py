"""Declarative protobuf (proto3 wire format) messages without protoc.

The reference gets protobuf classes from the TensorFlow Java jar and registers them with
Kryo (``LIB/util/RegistrationUtils.java:18-86``).  There is no protoc / TF in this
environment, so the TF message types we need are described here as field tables and
(de)serialized by a small generic codec.  The hot scan of length-delimited fields runs
in C++ (``_native.pb_scan``); a pure-Python fallback keeps the module importable before
the extension is built.

A message class declares ``FIELDS = [F(number, name, kind, ...)]``.  Kinds:
``int32 int64 uint32 uint64 sint32 sint64 bool enum float double fixed32 fixed64 string
bytes message map``.  Repeated scalars decode both packed and unpacked forms and encode
packed (proto3 default).
"""
from __future__ import annotations

import struct
from typing import Any, Callable

import numpy as np

try:  # the native scanner is optional at import time
    from .. import _ext

    _scan_native: Callable[[bytes], list] | None = None

    def _get_scan():
        global _scan_native
        if _scan_native is None:
            mod = _ext.native(required=False)
            _scan_native = mod.pb_scan if mod is not None else _scan_py
        return _scan_native

except Exception:  # pragma: no cover - defensive
    def _get_scan():
        return _scan_py


# ------------------------------------------------------------------------------ varints
def encode_varint(v: int) -> bytes:
    if v < 0:
        v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def decode_varint(buf: bytes, off: int) -> tuple[int, int]:
    r = 0
    shift = 0
    while True:
        if off >= len(buf):
            raise ValueError("truncated varint")
        c = buf[off]
        off += 1
        r |= (c & 0x7F) << shift
        if not c & 0x80:
            return r, off
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _scan_py(buf: bytes) -> list[tuple[int, int, Any]]:
    out = []
    off = 0
    n = len(buf)
    mv = memoryview(buf)
    while off < n:
        key, off = decode_varint(buf, off)
        field, wt = key >> 3, key & 7
        if wt == 0:
            v, off = decode_varint(buf, off)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, off)[0]
            off += 8
        elif wt == 2:
            ln, off = decode_varint(buf, off)
            if off + ln > n:
                raise ValueError("truncated length-delimited field")
            v = bytes(mv[off : off + ln])
            off += ln
        elif wt == 5:
            v = struct.unpack_from("<I", buf, off)[0]
            off += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.append((field, wt, v))
    return out


def scan(buf: bytes) -> list[tuple[int, int, Any]]:
    return _get_scan()(buf)


def _to_signed(v: int, bits: int) -> int:
    if v >= 1 << (bits - 1):
        v -= 1 << bits
    return v


def _zigzag_dec(v: int) -> int:
    return (v >> 1) ^ -(v & 1)


def _zigzag_enc(v: int) -> int:
    return (v << 1) ^ (v >> 63)


_VARINT_KINDS = {"int32", "int64", "uint32", "uint64", "sint32", "sint64", "bool", "enum"}
_FIXED32 = {"float": "<f", "fixed32": "<I", "sfixed32": "<i"}
_FIXED64 = {"double": "<d", "fixed64": "<Q", "sfixed64": "<q"}


class F:
    """A field descriptor."""

    __slots__ = ("number", "name", "kind", "repeated", "msg", "key_kind", "value_kind", "default")

    def __init__(self, number: int, name: str, kind: str, repeated: bool = False, msg: Any = None,
                 key_kind: str = "string", value_kind: str = "message"):
        self.number = number
        self.name = name
        self.kind = kind
        self.repeated = repeated
        self.msg = msg  # message class (or a zero-arg callable returning it, for recursion)
        self.key_kind = key_kind
        self.value_kind = value_kind
        if kind == "map":
            self.default = dict
        elif repeated:
            self.default = list
        elif kind == "message":
            self.default = lambda: None
        elif kind in ("string",):
            self.default = lambda: ""
        elif kind == "bytes":
            self.default = lambda: b""
        elif kind in ("float", "double"):
            self.default = lambda: 0.0
        elif kind == "bool":
            self.default = lambda: False
        else:
            self.default = lambda: 0

    def msg_cls(self):
        m = self.msg
        if m is not None and not isinstance(m, type):
            m = m()
        return m


def _decode_scalar(kind: str, wt: int, v: Any):
    if kind in _VARINT_KINDS:
        if kind == "bool":
            return bool(v)
        if kind in ("int32", "enum", "int64"):
            return _to_signed(v, 64)
        if kind == "sint32" or kind == "sint64":
            return _zigzag_dec(v)
        return v
    if kind in _FIXED32:
        if wt != 5:
            raise ValueError(f"field kind {kind} with wire type {wt}")
        return struct.unpack(_FIXED32[kind], struct.pack("<I", v))[0]
    if kind in _FIXED64:
        if wt != 1:
            raise ValueError(f"field kind {kind} with wire type {wt}")
        return struct.unpack(_FIXED64[kind], struct.pack("<Q", v))[0]
    if kind == "string":
        return v.decode("utf-8", errors="surrogateescape")
    if kind == "bytes":
        return v
    raise ValueError(kind)


def _decode_packed(kind: str, payload: bytes) -> list:
    if kind in _FIXED32:
        dt = {"float": "<f4", "fixed32": "<u4", "sfixed32": "<i4"}[kind]
        return np.frombuffer(payload, dtype=dt).tolist()
    if kind in _FIXED64:
        dt = {"double": "<f8", "fixed64": "<u8", "sfixed64": "<i8"}[kind]
        return np.frombuffer(payload, dtype=dt).tolist()
    out = []
    off = 0
    while off < len(payload):
        v, off = decode_varint(payload, off)
        out.append(_decode_scalar(kind, 0, v))
    return out


def _encode_scalar_payload(kind: str, v: Any) -> tuple[int, bytes]:
    """Returns (wire_type, bytes) for a single scalar value."""
    if kind in _VARINT_KINDS:
        if kind in ("sint32", "sint64"):
            v = _zigzag_enc(int(v))
        return 0, encode_varint(int(v))
    if kind in _FIXED32:
        return 5, struct.pack(_FIXED32[kind], v)
    if kind in _FIXED64:
        return 1, struct.pack(_FIXED64[kind], v)
    if kind == "string":
        b = v.encode("utf-8", errors="surrogateescape")
        return 2, encode_varint(len(b)) + b
    if kind == "bytes":
        b = bytes(v)
        return 2, encode_varint(len(b)) + b
    raise ValueError(kind)


def _key(number: int, wt: int) -> bytes:
    return encode_varint((number << 3) | wt)


class Message:
    """Base class for declarative protobuf messages."""

    FIELDS: list[F] = []
    _by_num: dict[int, F]
    _by_name: dict[str, F]

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        cls._by_num = {f.number: f for f in cls.FIELDS}
        cls._by_name = {f.name: f for f in cls.FIELDS}

    def __init__(self, **kw):
        for f in self.FIELDS:
            object.__setattr__(self, f.name, f.default())
        self._unknown: list[tuple[int, int, Any]] = []
        for k, v in kw.items():
            if k not in self._by_name:
                raise TypeError(f"{type(self).__name__} has no field {k!r}")
            setattr(self, k, v)

    # ------------------------------------------------------------------ decode
    @classmethod
    def decode(cls, buf: bytes | bytearray | memoryview):
        if not isinstance(buf, bytes):
            buf = bytes(buf)
        self = cls()
        for num, wt, v in scan(buf):
            f = cls._by_num.get(num)
            if f is None:
                self._unknown.append((num, wt, v))
                continue
            if f.kind == "map":
                kf = F(1, "k", f.key_kind)
                ent_k, ent_v = kf.default(), None
                for n2, wt2, v2 in scan(v):
                    if n2 == 1:
                        ent_k = _decode_scalar(f.key_kind, wt2, v2)
                    elif n2 == 2:
                        ent_v = f.msg_cls().decode(v2) if f.value_kind == "message" else _decode_scalar(f.value_kind, wt2, v2)
                if ent_v is None:
                    ent_v = f.msg_cls()() if f.value_kind == "message" else F(2, "v", f.value_kind).default()
                getattr(self, f.name)[ent_k] = ent_v
            elif f.kind == "message":
                m = f.msg_cls().decode(v)
                if f.repeated:
                    getattr(self, f.name).append(m)
                else:
                    object.__setattr__(self, f.name, m)
            elif f.repeated:
                lst = getattr(self, f.name)
                if wt == 2 and f.kind not in ("string", "bytes"):
                    lst.extend(_decode_packed(f.kind, v))
                else:
                    lst.append(_decode_scalar(f.kind, wt, v))
            else:
                object.__setattr__(self, f.name, _decode_scalar(f.kind, wt, v))
        return self

    # ------------------------------------------------------------------ encode
    def encode(self) -> bytes:
        out = bytearray()
        for f in self.FIELDS:
            val = getattr(self, f.name)
            if f.kind == "map":
                for k in sorted(val):
                    wt_k, pk = _encode_scalar_payload(f.key_kind, k)
                    ent = _key(1, wt_k) + pk
                    v = val[k]
                    if f.value_kind == "message":
                        b = v.encode()
                        ent += _key(2, 2) + encode_varint(len(b)) + b
                    else:
                        wt_v, pv = _encode_scalar_payload(f.value_kind, v)
                        ent += _key(2, wt_v) + pv
                    out += _key(f.number, 2) + encode_varint(len(ent)) + ent
            elif f.kind == "message":
                items = val if f.repeated else ([val] if val is not None else [])
                for m in items:
                    b = m.encode()
                    out += _key(f.number, 2) + encode_varint(len(b)) + b
            elif f.repeated:
                if not len(val):
                    continue
                if f.kind in ("string", "bytes"):
                    for x in val:
                        wt, p = _encode_scalar_payload(f.kind, x)
                        out += _key(f.number, wt) + p
                else:
                    if f.kind in _FIXED32 or f.kind in _FIXED64:
                        dt = {"float": "<f4", "fixed32": "<u4", "sfixed32": "<i4", "double": "<f8",
                              "fixed64": "<u8", "sfixed64": "<i8"}[f.kind]
                        p = np.asarray(val, dtype=dt).tobytes()
                    else:
                        p = b"".join(_encode_scalar_payload(f.kind, x)[1] for x in val)
                    out += _key(f.number, 2) + encode_varint(len(p)) + p
            else:
                if val == f.default() and not isinstance(val, Message):
                    continue  # proto3: default scalars are not emitted
                wt, p = _encode_scalar_payload(f.kind, val)
                out += _key(f.number, wt) + p
        for num, wt, v in self._unknown:  # round-trip unknown fields verbatim
            if wt == 0:
                out += _key(num, 0) + encode_varint(v)
            elif wt == 1:
                out += _key(num, 1) + struct.pack("<Q", v)
            elif wt == 2:
                out += _key(num, 2) + encode_varint(len(v)) + v
            elif wt == 5:
                out += _key(num, 5) + struct.pack("<I", v)
        return bytes(out)

    SerializeToString = encode

    @classmethod
    def FromString(cls, b: bytes):
        return cls.decode(b)

    # ------------------------------------------------------------------ helpers
    def __eq__(self, other):
        if type(self) is not type(other):
            return NotImplemented
        return all(getattr(self, f.name) == getattr(other, f.name) for f in self.FIELDS)

    def __repr__(self):
        parts = []
        for f in self.FIELDS:
            v = getattr(self, f.name)
            if v in (None, "", b"", 0, 0.0, False) or (isinstance(v, (list, dict)) and not v):
                continue
            if isinstance(v, bytes) and len(v) > 32:
                v = f"<{len(v)} bytes>"
            parts.append(f"{f.name}={v!r}")
        return f"{type(self).__name__}({', '.join(parts)})"

    def copy(self):
        return type(self).decode(self.encode())
