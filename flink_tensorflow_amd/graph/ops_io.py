"""I/O and string op kernels: ParseExample, DecodeJpeg/Png, string ops, SaveV2/RestoreV2.

* ``ParseExample`` runs the batched C++ parser (half_plus_two
  ``tf_example → x, x2``).
* ``SaveV2``/``RestoreV2``/``MergeV2Checkpoints``/``ShardedFilename``/``StringJoin`` are
  bound to the native bundle I/O (``io/bundle.py``) so that the SaverDef-driven
  save/restore in ``LIB/io/Saver.scala:55-89`` works on graphs exported by TF.
* ``DecodeJpeg`` decodes on the host with Pillow (no rocJPEG in the environment).
"""
from __future__ import annotations

import io as _io
import os

import numpy as np
import torch

from ..io import bundle
from ..types.dtypes import DataType
from ..types.example import BYTES, FLOAT, INT64, parse_example_dense, parse_example_varlen
from ..types.tensor import StringTensor
from .op_registry import register


def _strs(t) -> list[bytes]:
    if isinstance(t, StringTensor):
        return list(t.array.reshape(-1))
    raise TypeError("expected a STRING tensor")


def _str(t) -> str:
    v = _strs(t)
    if len(v) != 1:
        raise ValueError("expected a scalar STRING tensor")
    return v[0].decode()


# ------------------------------------------------------------------ ParseExample
@register("ParseExample")
def _parse_example(ctx, node, serialized, names, *rest):
    """TF ``ParseExample``: outputs ``sparse_indices[Nsparse]``, ``sparse_values[Nsparse]``,
    ``sparse_shapes[Nsparse]``, then ``dense_values[Ndense]``.  Sparse (``VarLenFeature``)
    keys come back as (indices [nnz, 2], values [nnz], dense_shape [2] = [N, max len])."""
    ns = node.attr("Nsparse", 0)
    nd = node.attr("Ndense", 0)
    sparse_keys = rest[:ns]
    dense_keys = rest[ns:ns + nd]
    dense_defaults = rest[ns + nd:]
    sparse_out: tuple = ()
    if ns:
        stypes = node.attr("sparse_types", []) or []
        sspecs = []
        for i in range(ns):
            dt = stypes[i]
            kind = FLOAT if dt == DataType.FLOAT else INT64 if dt == DataType.INT64 else BYTES
            sspecs.append((_strs(sparse_keys[i])[0].decode(), kind, dt))
        trip = parse_example_varlen(_strs(serialized), [(k, kind) for k, kind, _ in sspecs])
        idx = tuple(torch.from_numpy(t[0]).to(ctx.device) for t in trip)
        vals = tuple(StringTensor(v, (len(v),)) if kind == BYTES else torch.from_numpy(v).to(dt.torch).to(ctx.device)
                     for (_, kind, dt), (_, v, _) in zip(sspecs, trip))
        shp = tuple(torch.from_numpy(t[2]).to(ctx.device) for t in trip)
        sparse_out = idx + vals + shp
    tdense = node.attr("Tdense", []) or []
    shapes = node.attr("dense_shapes", []) or []
    specs = []
    for i in range(nd):
        key = _strs(dense_keys[i])[0].decode()
        dt = tdense[i]
        shp = shapes[i].as_list() if hasattr(shapes[i], "as_list") else list(shapes[i])
        numel = int(np.prod(shp)) if shp else 1
        dflt = dense_defaults[i]
        dflt_v = None
        if isinstance(dflt, torch.Tensor) and dflt.numel() > 0:
            dflt_v = dflt.detach().cpu().reshape(-1).double().numpy()
        elif isinstance(dflt, StringTensor) and dflt.numel() > 0:
            dflt_v = dflt.array.reshape(-1)
        kind = FLOAT if dt == DataType.FLOAT else INT64 if dt == DataType.INT64 else BYTES
        specs.append((key, kind, numel, dflt_v, dt, shp))
    ser = _strs(serialized)
    arrs = parse_example_dense(ser, [(k, kind, n, d) for k, kind, n, d, _, _ in specs]) if specs else []
    outs = list(sparse_out)
    for (k, kind, n, d, dt, shp), a in zip(specs, arrs):
        shape = (len(ser), *shp)
        if kind == BYTES:
            outs.append(StringTensor(a.reshape(-1), shape))
        else:
            outs.append(torch.from_numpy(a).reshape(shape).to(dt.torch).to(ctx.device))
    return tuple(outs)


@register("ParseSingleExample")
def _parse_single_example(ctx, node, serialized, *dense_defaults):
    keys = [k.decode() if isinstance(k, bytes) else k for k in (node.attr("dense_keys", []) or [])]
    tdense = node.attr("Tdense", []) or []
    shapes = node.attr("dense_shapes", []) or []
    specs = []
    for i, key in enumerate(keys):
        shp = shapes[i].as_list()
        n = int(np.prod(shp)) if shp else 1
        d = dense_defaults[i]
        dv = d.detach().cpu().reshape(-1).double().numpy() if isinstance(d, torch.Tensor) and d.numel() else None
        specs.append((key, FLOAT if tdense[i] == DataType.FLOAT else INT64, n, dv))
    arrs = parse_example_dense(_strs(serialized), specs)
    return tuple(torch.from_numpy(a).reshape(shapes[i].as_list()).to(tdense[i].torch).to(ctx.device)
                 for i, a in enumerate(arrs))


# ------------------------------------------------------------------ images
def decode_image_bytes(data: bytes, channels: int = 3) -> np.ndarray:
    from PIL import Image

    img = Image.open(_io.BytesIO(data))
    mode = {1: "L", 3: "RGB", 4: "RGBA"}.get(channels, None)
    if mode:
        img = img.convert(mode)
    arr = np.asarray(img, dtype=np.uint8)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    return arr


def fit_image_bytes(data: bytes, h: int, w: int) -> np.ndarray:
    """Pillow decode to RGB ``[h, w, 3]`` (bilinear resize when the file has another size):
    the fallback for what the native baseline decoder declines (progressive, PNG, ...)."""
    from PIL import Image

    img = Image.open(_io.BytesIO(data)).convert("RGB")
    if img.size != (w, h):
        img = img.resize((w, h), Image.BILINEAR)
    return np.asarray(img, dtype=np.uint8)


def decode_jpegs_into(ptr: int, nbytes: int, blobs: list, stride: int, h: int, w: int, threads: int = 8,
                      rows=None) -> int:
    """Decode ``blobs`` (JPEG byte strings) into consecutive ``stride``-byte rows at host
    address ``ptr`` as RGB ``[h, w, 3]`` uint8: the native baseline decoder on the host
    pool (``csrc/jpeg.cpp``, GIL released); every image it reports as not taken goes through
    :func:`fit_image_bytes`.  ``rows`` (indexable ``[n] -> writable [h, w, 3]``) receives the
    fallbacks; when None a numpy view over ``ptr`` is used.  Returns the fallback count."""
    from .. import _ext

    st = _ext.native().jpeg_decode_into(ptr, nbytes, blobs, stride, h, w, threads)
    bad = [k for k, code in enumerate(st) if code]
    if bad and rows is None:
        import ctypes

        buf = (ctypes.c_uint8 * (len(blobs) * stride)).from_address(ptr)
        rows = np.frombuffer(buf, np.uint8).reshape(len(blobs), stride)[:, : h * w * 3].reshape(-1, h, w, 3)
    for k in bad:
        img = fit_image_bytes(bytes(blobs[k]), h, w)
        if isinstance(rows, np.ndarray):
            rows[k] = img
        else:
            rows[k].copy_(__import__("torch").from_numpy(img))
    return len(bad)


def decode_rgb(data: bytes) -> np.ndarray:
    """One image file -> RGB ``[h, w, 3]`` uint8 at its own size: the native baseline decoder
    for baseline JPEGs (``csrc/jpeg.cpp``, GIL released), Pillow for everything else."""
    from .. import _ext

    nat = _ext.native()
    h, w, nc, baseline = nat.jpeg_info(bytes(data))
    if baseline and nc in (1, 3) and h > 0 and w > 0:
        out = np.empty((h, w, 3), np.uint8)
        if nat.jpeg_decode_into(out.ctypes.data, out.nbytes, [data], h * w * 3, h, w, 1)[0] == 0:
            return out
    return decode_image_bytes(bytes(data), 3)


def decode_jpegs(blobs: list, h: int, w: int, threads: int = 8) -> np.ndarray:
    """``[n, h, w, 3]`` uint8 from JPEG byte strings (see :func:`decode_jpegs_into`)."""
    out = np.empty((len(blobs), h, w, 3), np.uint8)
    if len(blobs):
        decode_jpegs_into(out.ctypes.data, out.nbytes, list(blobs), h * w * 3, h, w, threads, rows=out)
    return out


@register("DecodeJpeg", "DecodePng", "DecodeImage", "DecodeBmp")
def _decode_jpeg(ctx, node, contents):
    ch = node.attr("channels", 0) or 3
    return (torch.from_numpy(decode_image_bytes(_strs(contents)[0], ch).copy()),)


@register("EncodeJpeg")
def _encode_jpeg(ctx, node, image):
    from PIL import Image

    buf = _io.BytesIO()
    Image.fromarray(image.cpu().numpy().squeeze()).save(buf, format="JPEG", quality=node.attr("quality", 95))
    return (StringTensor(buf.getvalue()),)


# ------------------------------------------------------------------ strings
@register("StringJoin")
def _string_join(ctx, node, *xs):
    sep = node.attr_bytes("separator", b"")
    arrays = [x.array for x in xs]
    shape = np.broadcast(*arrays).shape if arrays else ()
    b = [np.broadcast_to(a, shape).reshape(-1) for a in arrays]
    out = [sep.join(parts) for parts in zip(*b)]
    return (StringTensor(out, shape),)


@register("ShardedFilename")
def _sharded_filename(ctx, node, basename, shard, num_shards):
    return (StringTensor(bundle.data_filename(_str(basename), int(shard.item()), int(num_shards.item()))
                         .replace(".data-", "-", 1).encode()),)


@register("ShardedFilespec")
def _sharded_filespec(ctx, node, basename, num_shards):
    return (StringTensor(f"{_str(basename)}-?????-of-{int(num_shards.item()):05d}".encode()),)


@register("StringToNumber")
def _string_to_number(ctx, node, x):
    dt = node.attr("out_type", DataType.FLOAT)
    return (torch.tensor([float(v) for v in _strs(x)], dtype=dt.torch).reshape(x.shape),)


@register("AsString")
def _as_string(ctx, node, x):
    return (StringTensor([str(v).encode() for v in x.reshape(-1).tolist()], tuple(x.shape)),)


# ------------------------------------------------------------------ checkpoints
@register("SaveV2")
def _save_v2(ctx, node, prefix, names, shape_and_slices, *tensors):
    """Whole tensors under their names; partitioned-variable slices (``shape_and_slices``
    ``"full shape start,len:..."``) as slice entries of the full variable."""
    p = _str(prefix)
    w = bundle.BundleWriter(p)
    vals = []
    for n, ss, t in zip(_strs(names), _strs(shape_and_slices), tensors):
        if hasattr(t, "read"):
            t = t.read()
        vals.append((n.decode(), ss.decode(), t))
    for n, ss, t in sorted(vals, key=lambda v: (v[0], v[1])):
        spec = bundle.parse_shape_and_slice(ss)
        if spec is None:
            w.add(n, t)
        else:
            w.add_slice(n, spec[0], spec[1], t)
    w.finish()
    return ()


@register("RestoreV2")
def _restore_v2(ctx, node, prefix, names, shape_and_slices):
    out = []
    with bundle.BundleReader(_str(prefix)) as r:
        for n, ss in zip(_strs(names), _strs(shape_and_slices)):
            spec = bundle.parse_shape_and_slice(ss.decode())
            if spec is None:
                out.append(r.read(n.decode(), device=ctx.device))
            else:
                e = r.entries.get(n.decode())
                if e is not None and [int(d) for d in (e.shape.as_list() or [])] != spec[0]:
                    raise ValueError(f"RestoreV2: {n.decode()!r} has shape {e.shape.as_list()}, slice spec says {spec[0]}")
                out.append(r.read_slice(n.decode(), spec[1], device=ctx.device))
    return tuple(out)


@register("MergeV2Checkpoints")
def _merge_v2(ctx, node, checkpoint_prefixes, destination_prefix):
    srcs = [s.decode() for s in _strs(checkpoint_prefixes)]
    bundle.merge_bundles(srcs, _str(destination_prefix), node.attr("delete_old_dirs", True))
    return ()


@register("ReadFile")
def _read_file(ctx, node, filename):
    with open(_str(filename), "rb") as f:
        return (StringTensor(f.read()),)


@register("WriteFile")
def _write_file(ctx, node, filename, contents):
    path = _str(filename)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(_strs(contents)[0])
    return ()
