"""Native baseline JPEG decoding into staging rows (``csrc/jpeg.cpp``
``jpeg_decode_into``) against Pillow's libjpeg: 4:2:0 / 4:2:2 / 4:4:4 chroma, restart
intervals, grayscale, odd sizes, quality 50-100; unsupported files (progressive, another
size, not a JPEG) are reported per image, never decoded wrongly.  Decoding is the
reference's ``DecodeJpeg`` of ``ImageNormalization.scala:42-77``."""
import io

import numpy as np
import pytest

from flink_tensorflow_amd import _ext


def _img(h, w, seed):
    from PIL import Image

    rng = np.random.default_rng(seed)
    low = rng.integers(0, 256, (max(2, h // 16), max(2, w // 16), 3), dtype=np.uint8)
    a = np.asarray(Image.fromarray(low).resize((w, h), Image.BICUBIC), np.float32)
    return np.clip(a + rng.normal(0, 12, a.shape), 0, 255).astype(np.uint8)


def _jpeg(a, **kw):
    from PIL import Image

    buf = io.BytesIO()
    Image.fromarray(a).save(buf, format="JPEG", **kw)
    return buf.getvalue()


def _pil(b):
    from PIL import Image

    return np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))


def _native(blobs, h, w, threads=4):
    out = np.zeros((len(blobs), h, w, 3), np.uint8)
    st = _ext.native().jpeg_decode_into(out.ctypes.data, out.nbytes, list(blobs), h * w * 3, h, w, threads)
    return out, st


@pytest.mark.parametrize("h,w,kw", [
    (256, 256, dict(quality=90)),                       # 4:2:0 (Pillow's default)
    (224, 240, dict(quality=75, subsampling=1)),        # 4:2:2
    (97, 131, dict(quality=95, subsampling=0)),         # 4:4:4, sizes not multiples of 8 / 16
    (64, 80, dict(quality=50)),
    (299, 299, dict(quality=100)),
])
def test_matches_pillow(h, w, kw):
    blobs = [_jpeg(_img(h, w, s), **kw) for s in range(6)]
    out, st = _native(blobs, h, w)
    assert st == [0] * len(blobs)
    ref = np.stack([_pil(b) for b in blobs]).astype(np.int16)
    d = np.abs(out.astype(np.int16) - ref)
    # float IDCT and triangle upsampling vs libjpeg's integer islow: a count or two apart
    assert d.max() <= 6 and d.mean() < 0.8, (d.max(), d.mean())


def test_restart_intervals_and_grayscale():
    from PIL import Image

    a = _img(120, 200, 3)
    # restart markers every few MCUs (Pillow forwards restart_marker_rows/blocks to libjpeg)
    b = _jpeg(a, quality=85, restart_marker_blocks=3)
    assert b.count(b"\xff\xd0") >= 1
    out, st = _native([b], 120, 200)
    assert st == [0]
    assert np.abs(out[0].astype(int) - _pil(b).astype(int)).max() <= 6
    g = io.BytesIO()
    Image.fromarray(a[..., 0]).save(g, format="JPEG", quality=90)
    out, st = _native([g.getvalue()], 120, 200)
    ref = _pil(g.getvalue())
    assert st == [0] and np.abs(out[0].astype(int) - ref.astype(int)).max() <= 4
    assert (out[0, ..., 0] == out[0, ..., 1]).all()


def test_unsupported_inputs_are_reported():
    a = _img(64, 64, 1)
    prog = _jpeg(a, quality=90, progressive=True)
    other = _jpeg(_img(32, 64, 2), quality=90)
    out, st = _native([prog, other, b"not a jpeg at all", _jpeg(a, quality=90)], 64, 64)
    assert st[:3] == [2, 4, 1] and st[3] == 0


def test_many_threads_same_result():
    blobs = [_jpeg(_img(128, 128, s), quality=90) for s in range(40)]
    a, _ = _native(blobs, 128, 128, threads=1)
    b, _ = _native(blobs, 128, 128, threads=16)
    assert np.array_equal(a, b)


def test_decode_jpegs_falls_back_to_pillow():
    from flink_tensorflow_amd.graph.ops_io import decode_jpegs

    a = _img(64, 64, 1)
    blobs = [_jpeg(a, quality=90, progressive=True), _jpeg(_img(32, 48, 2), quality=90), _jpeg(a, quality=90)]
    out = decode_jpegs(blobs, 64, 64, threads=2)
    assert np.abs(out[0].astype(int) - _pil(blobs[0]).astype(int)).max() <= 6  # progressive: Pillow
    from PIL import Image

    ref1 = np.asarray(Image.open(io.BytesIO(blobs[1])).convert("RGB").resize((64, 64), Image.BILINEAR))
    assert np.array_equal(out[1], ref1)  # another size: Pillow + bilinear resize
    assert np.abs(out[2].astype(int) - _pil(blobs[2]).astype(int)).max() <= 6


def test_deferred_decode_job_matches_decoded_records(tmp_path):
    """``ImageInputFormat(defer_decode=True)`` carries the file bytes; the image model
    decodes them (native pool) -- same labels as the records decoded in the reader."""
    from flink_tensorflow_amd.models.zoo.image_classifier import ResNet50Model
    from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat

    blobs = [_jpeg(_img(64, 64, s), quality=95) for s in range(3)]
    for i, b in enumerate(blobs):
        (tmp_path / f"im{i}.jpg").write_bytes(b)
    deferred = ImageInputFormat(defer_decode=True)
    eager = ImageInputFormat()
    recs_d = [deferred.read_record(f"im{i}.jpg", b) for i, b in enumerate(blobs)]
    recs_e = [eager.read_record(f"im{i}.jpg", b) for i, b in enumerate(blobs)]
    assert all(isinstance(r[1], bytes) for r in recs_d)
    m = ResNet50Model(image_hw=(64, 64), buckets=(4,), depth_layers=26, device="cpu")
    m.open()
    try:
        ld = m.label(recs_d)
        # the reference decoder path (Pillow) vs the native one differ by a count or two per
        # pixel; the top-1 class must agree
        le = m.label([(n, _native([b], 64, 64)[0][0]) for (n, _), b in zip(recs_e, blobs)])
        assert [r[0][1] for r in ld] == [r[0][1] for r in le]
        assert np.allclose([r[0][0] for r in ld], [r[0][0] for r in le], rtol=1e-5)
    finally:
        m.close()


def test_chained_reader_bulk_run_matches_per_record(tmp_path):
    """The chained file reader's bulk path (``process_batch``: the run's files read by the
    native pool, one ``emit_many`` into the consumer's ``process_many``) yields the same
    records, in order, as the per-record path; an unreadable file still raises."""
    from flink_tensorflow_amd.models.zoo.inception import ImageInputFormat
    from flink_tensorflow_amd.runtime.operators import ChainOperator, FileReaderOperator, Operator, Record

    blobs = [_jpeg(_img(32, 32, s), quality=90) for s in range(7)]
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"f{i}.jpg"
        p.write_bytes(b)
        paths.append(str(p))

    class Sink(Operator):
        def __init__(self):
            super().__init__(None, "sink")
            self.got, self.runs = [], 0

        def process(self, rec, input_index=0):
            self.got.append(rec.value)

        def process_many(self, values, ts=None):
            self.runs += 1
            self.got.extend(values)

    def run(bulk):
        sink = Sink()
        chain = ChainOperator([FileReaderOperator(ImageInputFormat(defer_decode=True)), sink])
        from flink_tensorflow_amd.runtime.operators import Output

        chain.setup(None, Output(lambda r: None))
        recs = [Record(p, 0.0) for p in paths]
        if bulk:
            chain.process_batch(recs, 0)
        else:
            for r in recs:
                chain.process(r, 0)
        return sink

    a, b = run(False), run(True)
    assert a.got == b.got and [n for n, _ in b.got] == [f"f{i}.jpg" for i in range(7)]
    assert b.runs == 1 and a.runs == 0
    assert [d for _, d in b.got] == blobs
    sink_chain = ChainOperator([FileReaderOperator(ImageInputFormat(defer_decode=True)), Operator(None, "x")])
    from flink_tensorflow_amd.runtime.operators import Output

    sink_chain.setup(None, Output(lambda r: None))
    with pytest.raises(FileNotFoundError):
        sink_chain.process_batch([Record(str(tmp_path / "missing.jpg"), 0.0)], 0)


@pytest.mark.gpu
@pytest.mark.parametrize("async_decode", [True, False])
def test_runner_decodes_jpeg_payloads_gpu(async_decode):
    """JPEG byte strings through the compiled ResNet operator's runner: decoded by the
    native pool into the pinned slot (in the background when ``async_decode``: launched by
    the next submit / drain), a progressive file through Pillow — the same top-k as the
    records decoded on the host first."""
    import numpy as np
    import torch

    from flink_tensorflow_amd.graph.ops_io import decode_jpegs
    from flink_tensorflow_amd.models.zoo.image_classifier import ResNet50Model

    blobs = [_jpeg(_img(64, 64, s), quality=90) for s in range(11)]
    blobs.append(_jpeg(_img(64, 64, 99), quality=90, progressive=True))
    m = ResNet50Model(image_hw=(64, 64), buckets=(8,), depth_layers=26, lanes=1)
    m.open()
    try:
        m._runner.async_decode = async_decode
        dec = decode_jpegs(blobs, 64, 64)

        def run(recs):
            out = []
            for lo in range(0, len(recs), 6):  # 6-record batches (bucket 8: padded)
                chunk = recs[lo:lo + 6]
                for res, _, _ in m.submit(chunk, np.zeros(len(chunk)), list(range(lo, lo + len(chunk)))):
                    out += res
            for res, _, _ in m.drain():
                out += res
            return out

        got = run([(f"f{i}.jpg", b) for i, b in enumerate(blobs)])
        ref = run([(f"f{i}.jpg", d) for i, d in enumerate(dec)])
        assert len(got) == len(ref) == len(blobs)
        assert got == ref  # identical staged bytes -> identical replays
        assert m._runner.decode_fallbacks >= 1
        torch.cuda.synchronize()
    finally:
        m.close()


def test_decode_rgb_any_size_and_fallbacks():
    """``decode_rgb`` (ImageInputFormat's decode): the native decoder at the file's own size
    for baseline JPEGs, Pillow for progressive files and PNGs."""
    from PIL import Image

    from flink_tensorflow_amd import _ext
    from flink_tensorflow_amd.graph.ops_io import decode_rgb

    a = _img(77, 123, 5)
    b = _jpeg(a, quality=92)
    assert _ext.native().jpeg_info(b) == (77, 123, 3, True)
    out = decode_rgb(b)
    assert out.shape == (77, 123, 3) and np.abs(out.astype(int) - _pil(b).astype(int)).max() <= 6
    prog = _jpeg(a, quality=92, progressive=True)
    assert _ext.native().jpeg_info(prog)[3] is False
    assert np.array_equal(decode_rgb(prog), _pil(prog))
    png = io.BytesIO()
    Image.fromarray(a).save(png, format="PNG")
    assert _ext.native().jpeg_info(png.getvalue()) == (0, 0, 0, False)
    assert np.array_equal(decode_rgb(png.getvalue()), a)
