"""Drives every entry point of the host runtime library (`_native`) with threads — run
under AddressSanitizer+UBSan or ThreadSanitizer by tests/test_sanitizers.py.  Loads the
library straight from FTM_NATIVE_LIB (no torch, no package import) so only the
instrumented code and the interpreter are in the process."""
import importlib.util
import os
import sys
import threading

import numpy as np

spec = importlib.util.spec_from_file_location("_native", os.environ["FTM_NATIVE_LIB"])
N = importlib.util.module_from_spec(spec)
spec.loader.exec_module(N)

rng = np.random.default_rng(0)

# CRC32C (known vector) and masked form
assert N.crc32c(b"123456789") == 0xE3069283
N.crc32c_masked(b"x" * 1000)

# TensorValue framing round trips
for shape in ([], [3], [2, 5, 7]):
    payload = rng.standard_normal(int(np.prod(shape)) if shape else 1).astype(np.float32).tobytes()
    enc = N.tv_encode(1, shape, payload)
    dt, sh, pl, nxt = N.tv_decode(enc, 0)
    assert dt == 1 and list(sh) == shape and pl == payload and nxt == len(enc)
    N.tv_copy(enc, 0)
many = N.tv_encode_many([(3, [4], np.arange(4, dtype=np.int32).tobytes()), (1, [], b"\0\0\0\0")])
assert len(N.tv_decode_many(many)) == 2
for bad in (b"", b"\x01\x00", many[:-3]):
    try:
        N.tv_decode(bad, 0)
    except Exception:
        pass

# protobuf helpers
N.pb_scan(b"\x08\x96\x01\x12\x03abc\x1d\x00\x00\x80\x3f")
vals = np.array([0, 1, -1, 300, 2 ** 40], dtype=np.int64)
assert list(N.pb_packed_varints(N.pb_encode_varints(vals), False)) == list(vals)

# tf.Example encode + multithreaded parse
x = rng.standard_normal((257, 3)).astype(np.float32)
ser = N.encode_float_examples(["x"], [x])
out = N.parse_examples(list(ser), [("x", 0, 3, None)], 8)
assert np.allclose(out[0], x)

# STRING tensors
elems = [b"", b"a", b"hello" * 50]
assert N.string_tensor_unpack(N.string_tensor_pack(elems), len(elems)) == elems

# SSTable build/parse with CRC verification
items = [(f"key{i:05d}".encode(), bytes(rng.integers(0, 256, i % 300, dtype=np.uint8))) for i in range(2000)]
tab = N.sstable_build(items, 4096, 16)
assert N.sstable_parse(tab, True) == items
corrupt = bytearray(tab)
corrupt[100] ^= 0xFF
try:
    N.sstable_parse(bytes(corrupt), True)
except Exception:
    pass

# staging gather from several Python threads at once
dst = np.zeros(64 * 4096, dtype=np.uint8)
recs = [bytes([i % 251]) * 3000 for i in range(64)]


def gather(k):
    for _ in range(20):
        d = np.zeros(64 * 4096, dtype=np.uint8)
        N.gather_into(d.ctypes.data, d.nbytes, recs, 4096, 4)
        assert d[4096 * 5] == 5


ts = [threading.Thread(target=gather, args=(k,)) for k in range(4)]
for t in ts:
    t.start()
for t in ts:
    t.join()

# the persistent copy pool (CopyPool in csrc/native.cpp) driven by two runner-like threads
# at once: micro-batches of 196 KB records (above the 1 MiB single-thread cut-off) gathered
# into staging slots in 64-record pieces with 8 helper threads each, while a third thread
# scatters records into a slab — concurrent jobs on one pool (round-3 driver abort suspect)
big = [np.full(196608, i % 251, dtype=np.uint8) for i in range(64)]
errors = []


def runner(k):
    try:
        slot = np.empty(64 * 196608, dtype=np.uint8)
        for it in range(12):
            for lo in range(0, 64, 16):
                N.gather_into(slot.ctypes.data + lo * 196608, slot.nbytes - lo * 196608, big[lo:lo + 16], 196608, 8)
            v = slot.reshape(64, 196608)
            if not all(v[i, 0] == i % 251 and v[i, -1] == i % 251 for i in range(64)):
                errors.append(f"runner {k} iteration {it}: wrong bytes")
    except Exception as e:  # noqa: BLE001
        errors.append(repr(e))


def scatterer():
    try:
        slab = np.empty(32 * 196608, dtype=np.uint8)
        offs = [i * 196608 for i in range(32)]
        for it in range(12):
            N.scatter_into(slab.ctypes.data, slab.nbytes, offs, big[:32], 4)
            if slab[5 * 196608] != 5:
                errors.append(f"scatter iteration {it}: wrong bytes")
    except Exception as e:  # noqa: BLE001
        errors.append(repr(e))


ts = [threading.Thread(target=runner, args=(k,)) for k in range(2)] + [threading.Thread(target=scatterer)]
for t in ts:
    t.start()
for t in ts:
    t.join()
assert not errors, errors
print("native exercise ok")
sys.stdout.flush()
