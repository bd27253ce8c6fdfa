"""SavedModel / bundle / executor conformance on the half_plus_two fixture.

Acceptance from SURVEY §7.2 step 1-2: the §2.9 facts (5 signatures, SaverDef, variables
a/b/c = 0.5/2/3), a byte-identical bundle round trip, all 5 signatures executing, and the
``DefaultSaverITCase`` save → mutate → restore sequence
(``TST/.../io/DefaultSaverITCase.scala:21-53``).
"""
import os
import shutil

import pytest
import torch

from flink_tensorflow_amd.io import bundle
from flink_tensorflow_amd.io.saver import DefaultSaver, Saver, VariableSaver
from flink_tensorflow_amd.models import (ClassificationMethod, PredictMethod, RegressionMethod, SavedModelModel,
                                         SignatureConstants, TensorFlowModel)
from flink_tensorflow_amd.types import example, feature


def test_metagraph_facts(half_plus_two):
    m = SavedModelModel(half_plus_two)
    mg = m.metagraph
    assert list(mg.meta_info_def.tags) == ["serve"]
    assert sorted(mg.signature_def) == ["classify_x_to_y", "regress_x2_to_y3", "regress_x_to_y", "regress_x_to_y2",
                                        "serving_default"]
    sd = mg.saver_def
    assert (sd.filename_tensor_name, sd.save_tensor_name, sd.restore_op_name) == (
        "save/Const:0", "save/Identity:0", "save/restore_all")
    assert sd.max_to_keep == 5 and sd.sharded and sd.version == 2
    assert mg.signature_def["regress_x_to_y"].method_name == SignatureConstants.REGRESS_METHOD_NAME
    assert not m.is_open  # metagraph did not load the bundle (B7)


def test_bundle_reads_variables(half_plus_two):
    r = bundle.BundleReader(os.path.join(half_plus_two, "variables", "variables"))
    vals = {k: float(v) for k, v in r.read_all().items()}
    assert vals == {"a": 0.5, "b": 2.0, "c": 3.0}


def test_bundle_roundtrip_byte_identical(half_plus_two, tmp_path):
    src = os.path.join(half_plus_two, "variables", "variables")
    t = bundle.BundleReader(src).read_all()
    dst = str(tmp_path / "v")
    bundle.save_tensors(dst, t)
    for suffix in (".index", ".data-00000-of-00001"):
        assert open(src + suffix, "rb").read() == open(dst + suffix, "rb").read()


def test_bundle_detects_corruption(tmp_path):
    p = str(tmp_path / "ck")
    bundle.save_tensors(p, {"w": torch.arange(16, dtype=torch.float32), "s": __import__(
        "flink_tensorflow_amd").types.StringTensor([b"ab", b"c"], (2,))})
    assert bundle.BundleReader(p).read("s").tolist() == [b"ab", b"c"]
    data = bytearray(open(p + ".data-00000-of-00001", "rb").read())
    data[3] ^= 0xFF
    open(p + ".data-00000-of-00001", "wb").write(bytes(data))
    with pytest.raises(bundle.DataLossError):
        bundle.BundleReader(p).read_all()
    idx = bytearray(open(p + ".index", "rb").read())
    idx[2] ^= 0xFF
    open(p + ".index", "wb").write(bytes(idx))
    with pytest.raises(bundle.DataLossError):
        bundle.BundleReader(p)


def _py_crc32c(data: bytes, crc: int = 0) -> int:
    """Bitwise CRC-32C (Castagnoli), independent of the native SSE4.2 implementation."""
    crc ^= 0xFFFFFFFF
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (0x82F63B78 if crc & 1 else 0)
    return crc ^ 0xFFFFFFFF


def _py_mask(crc: int) -> int:
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def test_string_tensor_entry_crc_follows_tf_layout(tmp_path):
    """Hand-built fixture of TF's ``WriteStringTensor`` layout: the entry CRC covers u32
    lengths + the stored (masked) length checksum + bytes, not the varint payload."""
    import struct

    from flink_tensorflow_amd.types import StringTensor

    elems = [b"hello", b"", b"x" * 200]
    fixed = b"".join(struct.pack("<I", len(e)) for e in elems)
    cks = struct.pack("<I", _py_mask(_py_crc32c(fixed)))
    varints = bytes([5, 0]) + bytes([200 & 0x7F | 0x80, 200 >> 7])
    want_payload = varints + cks + b"".join(elems)
    want_crc = _py_mask(_py_crc32c(b"".join(elems), _py_crc32c(cks, _py_crc32c(fixed))))
    p = str(tmp_path / "s")
    bundle.save_tensors(p, {"s": StringTensor(elems, (3,))})
    assert open(p + ".data-00000-of-00001", "rb").read() == want_payload
    r = bundle.BundleReader(p)
    assert r.entries["s"].crc32c == want_crc
    assert r.read("s").tolist() == elems


class HalfPlusTwo(TensorFlowModel):
    """``TST/.../ml/HalfPlusTwo.scala:14-28``."""

    def __init__(self, path):
        super().__init__(device="cpu")
        self._loader = TensorFlowModel.load(path, "serve")

    @property
    def loader(self):
        return self._loader

    def regress_x_to_y(self, x):
        return self.function("regress_x_to_y", RegressionMethod()).apply(x)

    def regress_x_to_y2(self, x):
        return self.function("regress_x_to_y2", RegressionMethod()).apply(x)


@pytest.fixture
def model(half_plus_two):
    m = HalfPlusTwo(half_plus_two)
    m.open()
    yield m
    m.close()


def test_all_five_signatures(model):
    exs = [example(("x", feature(float(v))), ("x2", feature(float(v) * 10))) for v in range(4)]
    y = model.regress_x_to_y(exs)
    assert y.reshape(-1).tolist() == [2.0, 2.5, 3.0, 3.5]
    assert model.regress_x_to_y2(exs).reshape(-1).tolist() == [3.0, 3.5, 4.0, 4.5]
    y3 = model.function("regress_x2_to_y3", RegressionMethod()).apply(torch.tensor([[2.0], [4.0]]))
    assert y3.reshape(-1).tolist() == [4.0, 5.0]
    classes, scores = model.function("classify_x_to_y", ClassificationMethod()).apply(exs)
    assert classes is None and scores.reshape(-1).tolist() == [2.0, 2.5, 3.0, 3.5]
    out = model.function("serving_default", PredictMethod()).apply({"x": torch.tensor([[1.0]])})
    assert out["y"].item() == 2.5
    # x2 default (0.0) is applied when the feature is absent
    exs_no_x2 = [example(("x", feature(1.0)))]
    y3b = model.session().run("y3:0", {"tf_example:0": __import__("flink_tensorflow_amd").types.messages_to_tensor(exs_no_x2)})
    assert y3b.item() == 3.0


def test_model_function_context_manager_and_metadata(model):
    fn = model.function("regress_x_to_y", RegressionMethod())
    with fn([example(("x", feature(2.0)))]) as y:
        assert y.item() == 3.0
    out, md = fn.run([example(("x", feature(2.0)))], run_metadata=True)
    names = [s.node_name for s in md.step_stats.dev_stats[0].node_stats]
    assert "ParseExample/ParseExample" in names and "y" in names


def test_method_name_mismatch_rejected(model):
    with pytest.raises(ValueError):
        model.function("serving_default", RegressionMethod())


def test_double_open_rejected(model):
    with pytest.raises(RuntimeError):
        model.open()


def _get_a(sess):
    return sess.run("a:0").item()


def _set_a(sess, v):
    sess.run(targets=["a/Assign"], feed_dict={"a/initial_value:0": torch.tensor(v)})


def test_default_saver_itcase(model, tmp_path):
    """save(a=1) → set a=2 → restore → a == 1."""
    sess = model.session()
    saver = Saver.create(model.metagraph.saver_def)
    assert isinstance(saver, DefaultSaver)
    _set_a(sess, 1.0)
    path = saver.save(sess, str(tmp_path / "model-0"))
    assert path == str(tmp_path / "model-0")
    assert os.path.exists(path + ".index") and os.path.exists(path + ".data-00000-of-00001")
    _set_a(sess, 2.0)
    assert _get_a(sess) == 2.0
    saver.restore(sess, path)
    assert _get_a(sess) == 1.0
    # the temp shard dir of the sharded saver was merged away
    assert not [d for d in os.listdir(tmp_path) if "_temp_" in d]


def test_variable_saver(model, tmp_path):
    sess = model.session()
    vs = VariableSaver()
    p = vs.save(sess, str(tmp_path / "vars"))
    _set_a(sess, 9.0)
    vs.restore(sess, p)
    assert _get_a(sess) == 0.5


def test_remote_fs_model_copy(half_plus_two):
    from flink_tensorflow_amd.utils import fs

    memfs = fs.get_fs("mem://x")[0]
    for root, _, files in os.walk(half_plus_two):
        for f in files:
            full = os.path.join(root, f)
            memfs.write_bytes("mem://models/hp2/" + os.path.relpath(full, half_plus_two), open(full, "rb").read())
    m = SavedModelModel("mem://models/hp2", device="cpu")
    assert "regress_x_to_y" in m.metagraph.signature_def
    m.open()
    try:
        y = m.function("regress_x_to_y", RegressionMethod()).apply([example(("x", feature(4.0)))])
        assert y.item() == 4.0
    finally:
        m.close()


def test_pickled_model_is_a_descriptor(model):
    import pickle

    m2 = pickle.loads(pickle.dumps(model))
    assert not m2.is_open
    m2.open()
    assert m2.regress_x_to_y([example(("x", feature(0.0)))]).item() == 2.0
    m2.close()


def test_asset_init_op_ran(model):
    v = model.session().variables["filename_tensor"]
    assert v.item() == b"foo.txt"


def teardown_module(module):
    shutil.rmtree("/tmp/ftm-none", ignore_errors=True)


def test_snapshot_writes_variables_only_when_changed(half_plus_two, tmp_path):
    """A read-only model writes nothing at a checkpoint; a changed one writes its bundle;
    an unchanged-since-last-bundle one hard-links that bundle (no D2H, no rewrite)."""
    import os
    from types import SimpleNamespace

    import torch

    from flink_tensorflow_amd.models import SavedModelModel

    m = SavedModelModel(half_plus_two, device="cpu")
    m.open()

    def snap(i):
        ctx = SimpleNamespace(checkpoint_dir=str(tmp_path / f"chk-{i}"), subtask_index=0)
        m.snapshot_state(ctx)
        return str(tmp_path / f"chk-{i}" / "models")

    d1 = snap(1)
    assert not any(f.startswith("variables") for _, _, fs in os.walk(d1) for f in fs)  # pristine: nothing
    m.session().run(targets=["a/Assign"], feed_dict={"a/initial_value:0": torch.tensor(3.0)})
    d2 = snap(2)
    idx2 = [os.path.join(r, f) for r, _, fs in os.walk(d2) for f in fs if f.endswith(".index")]
    assert len(idx2) == 1
    d3 = snap(3)
    idx3 = [os.path.join(r, f) for r, _, fs in os.walk(d3) for f in fs if f.endswith(".index")]
    assert len(idx3) == 1 and os.path.samefile(idx2[0], idx3[0])  # linked, not rewritten
    # a restore from the linked bundle gives the changed value
    m2 = SavedModelModel(half_plus_two, device="cpu")
    m2.open()
    m2.restore_variables(idx3[0][: -len(".index")])
    assert float(m2.session().variables["a"]) == 3.0
    m.close()
    m2.close()


def test_function_cache_accepts_unhashable_options(half_plus_two):
    """``batch_buckets`` as a list (what YAML / ``config.to_dict()`` produce) still caches."""
    from flink_tensorflow_amd.models import PredictMethod, SavedModelModel

    m = SavedModelModel(half_plus_two, device="cpu")
    m.open()
    f1 = m.function("serving_default", PredictMethod(), batch_buckets=[1, 4])
    f2 = m.function("serving_default", PredictMethod(), batch_buckets=[1, 4])
    assert f1 is f2
    m.close()


# ------------------------------------------------------------------ multi-shard / partitioned checkpoints
def test_two_shard_bundle_roundtrip_and_merge(tmp_path):
    """A hand-built 2-shard bundle reads back; MergeV2Checkpoints of it plus a 1-shard
    bundle renames all three data shards under the destination with remapped shard ids."""
    a, b, c = torch.arange(12, dtype=torch.float32).reshape(3, 4), torch.tensor([1, 2, 3], dtype=torch.int64), \
        torch.full((2, 2), 7.5)
    p2 = str(tmp_path / "two" / "ckpt")
    w0 = bundle.BundleWriter(p2, 0, 2)
    w0.add("a", a)
    w1 = bundle.BundleWriter(p2, 1, 2)
    w1.add("b", b)
    entries = {**w0.finish(write_index=False), **w1.finish(write_index=False)}
    bundle.write_index_file(p2, entries, 2)
    with bundle.BundleReader(p2) as r:
        assert r.header.num_shards == 2 and r.keys() == ["a", "b"]
        assert torch.equal(r.read("a"), a) and torch.equal(r.read("b"), b)
    p1 = str(tmp_path / "one" / "ckpt")
    bundle.save_tensors(p1, {"c": c})
    dst = str(tmp_path / "merged" / "model")
    bundle.merge_bundles([p2, p1], dst)
    with bundle.BundleReader(dst) as r:
        assert r.header.num_shards == 3
        assert sorted(e.shard_id for e in r.entries.values()) == [0, 1, 2]
        assert torch.equal(r.read("a"), a) and torch.equal(r.read("b"), b) and torch.equal(r.read("c"), c)
    assert not os.path.exists(p2 + ".index") and not os.path.exists(p1 + ".index")


def test_partitioned_variable_slices_roundtrip(tmp_path):
    """SaveV2 / RestoreV2 with ``shape_and_slices``: a [6, 4] variable saved as two row
    partitions (full-tensor entry with the slice list + one ordered-code key per slice)
    restores whole, per partition and across the partition boundary."""
    from types import SimpleNamespace

    import flink_tensorflow_amd.graph.ops_io  # noqa: F401  (registers the checkpoint ops)
    from flink_tensorflow_amd.graph.op_registry import lookup as get_op
    from flink_tensorflow_amd.types.tensor import StringTensor

    full = torch.arange(24, dtype=torch.float32).reshape(6, 4)
    prefix = str(tmp_path / "part" / "ckpt")
    ctx = SimpleNamespace(device=torch.device("cpu"))
    save, restore = get_op("SaveV2"), get_op("RestoreV2")
    save(ctx, None, StringTensor(prefix), StringTensor(["w", "w", "v"]),
         StringTensor(["6 4 0,2:-", "6 4 2,4:-", ""]), full[:2], full[2:], torch.ones(3))
    with bundle.BundleReader(prefix) as r:
        assert r.keys() == ["v", "w"]
        e = r.entries["w"]
        assert e.shape.as_list() == [6, 4] and len(e.slices) == 2
    got = restore(ctx, None, StringTensor(prefix), StringTensor(["w", "w", "w", "v"]),
                  StringTensor(["", "6 4 1,3:-", "6 4 0,6:1,2", ""]))
    # a whole-tensor read of a partitioned variable assembles it from its slices
    assert torch.equal(got[1], full[1:4]) and torch.equal(got[2], full[:, 1:3]) and torch.equal(got[3], torch.ones(3))


def test_ordered_code_slice_keys_sort_like_tf():
    """The slice keys are order-preserving in (start, length), and small / large / negative
    numbers take the TF encoding lengths (1 byte below 64, 2 bytes from 64, -1 = 0x7f)."""
    k = bundle._ordered_signed_increasing
    assert k(0) == b"\x80" and k(5) == b"\x85" and k(-1) == b"\x7f" and len(k(64)) == 2 and len(k(8191)) == 2
    assert len(k(8192)) == 3
    vals = [-70000, -65, -64, -1, 0, 1, 63, 64, 100, 8191, 8192, 1 << 40]
    enc = [k(v) for v in vals]
    assert enc == sorted(enc)


@pytest.mark.gpu
def test_bundle_reads_into_hbm_through_pinned_staging_gpu(tmp_path):
    """Checkpoint reads with a CUDA device go file -> pinned ring -> HBM (chunked: a 80 MB
    tensor crosses the 32 MB staging chunks) with the checksum verified on the way."""
    big = torch.randn(20 << 20)  # 80 MB fp32
    small = torch.arange(10, dtype=torch.int32)
    prefix = str(tmp_path / "ck")
    bundle.save_tensors(prefix, {"big": big, "small": small})
    dev = torch.device("cuda", 0)
    with bundle.BundleReader(prefix) as r:
        g = r.read("big", device=dev)
        s = r.read("small", device=dev)
        torch.cuda.synchronize()
    assert g.device.type == "cuda" and torch.equal(g.cpu(), big) and torch.equal(s.cpu(), small)
    data = bundle.data_filename(prefix, 0, 1)
    raw = bytearray(open(data, "rb").read())
    raw[1000] ^= 0xFF
    open(data, "wb").write(bytes(raw))
    with bundle.BundleReader(prefix) as r:
        with pytest.raises(bundle.DataLossError):
            r.read("big", device=dev)
    # an entry whose stored size disagrees with its shape fails loudly (the CRC alone covers
    # only the stored bytes: the device tensor's tail would stay uninitialised)
    bundle.save_tensors(prefix, {"big": big, "small": small})
    with bundle.BundleReader(prefix) as r:
        r.entries["small"].size -= 4
        with pytest.raises(bundle.DataLossError, match="needs"):
            r.read("small", device=dev)


def test_merge_rejects_partitions_that_disagree_on_the_full_shape(tmp_path):
    """MergeV2Checkpoints of two shards holding slices of one partitioned variable whose
    full shapes disagree is an error (TF rejects it too)."""
    from types import SimpleNamespace

    import flink_tensorflow_amd.graph.ops_io  # noqa: F401  (registers the checkpoint ops)
    from flink_tensorflow_amd.graph.op_registry import lookup as get_op
    from flink_tensorflow_amd.types.tensor import StringTensor

    ctx = SimpleNamespace(device=torch.device("cpu"))
    save = get_op("SaveV2")
    p0, p1 = str(tmp_path / "s0" / "ckpt"), str(tmp_path / "s1" / "ckpt")
    save(ctx, None, StringTensor(p0), StringTensor(["w"]), StringTensor(["6 4 0,2:-"]), torch.ones(2, 4))
    save(ctx, None, StringTensor(p1), StringTensor(["w"]), StringTensor(["8 4 2,4:-"]), torch.ones(4, 4))
    with pytest.raises(ValueError, match="disagree"):
        bundle.merge_bundles([p0, p1], str(tmp_path / "m" / "ckpt"))
