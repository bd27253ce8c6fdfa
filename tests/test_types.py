"""L3 types: TensorValue framing, dtypes, TensorName, STRING packing, injections.

Reference tests mirrored: ``TST/.../types/TensorValueTest.java`` (2x3 int32 round trips),
``TST/.../types/TensorInjectionsTest.scala`` (Example <-> tensor), ``TST/.../ArraysTest.scala``.
"""
import io
import pickle
import struct

import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from flink_tensorflow_amd.types import (DataType, StringTensor, TensorInjections, TensorName, TensorValue,
                                        TypedTensor, VersionMismatchException, array_to_tensor, example, feature,
                                        get_data_type, get_value, messages_to_tensor, tagged_as, tensor_to_array,
                                        tensor_to_messages)
from flink_tensorflow_amd.proto.messages import Example


def test_tensor_value_from_tensor_2x3_int32():
    t = torch.tensor([[1, 2, 3], [4, 5, 6]], dtype=torch.int32)
    v = TensorValue.from_tensor(t)
    assert v.dtype == DataType.INT32
    assert v.shape() == (2, 3)
    assert v.to_tensor().reshape(-1).tolist() == [1, 2, 3, 4, 5, 6]


def test_framing_layout_is_reference_compatible():
    v = TensorValue.from_tensor(torch.tensor([1.5, 2.5], dtype=torch.float32))
    b = v.to_bytes()
    # u8 version | i32 dtype | i32 rank | i64 dims | i32 nbytes | payload (native order)
    assert b[0] == 1
    assert struct.unpack(">i", b[1:5])[0] == 1
    assert struct.unpack(">i", b[5:9])[0] == 1
    assert struct.unpack(">q", b[9:17])[0] == 2
    assert struct.unpack(">i", b[17:21])[0] == 8
    assert struct.unpack("<2f", b[21:29]) == (1.5, 2.5)
    assert len(b) == v.binary_length() == 1 + 4 + 4 + 8 + 4 + 8


def test_version_mismatch():
    b = bytearray(TensorValue.from_tensor(torch.zeros(2)).to_bytes())
    b[0] = 2
    with pytest.raises(VersionMismatchException):
        TensorValue.from_bytes(bytes(b))


_dtypes = st.sampled_from([torch.float32, torch.float64, torch.int32, torch.int64, torch.uint8, torch.bool,
                           torch.bfloat16, torch.float16, torch.int8])


@settings(max_examples=60, deadline=None)
@given(dt=_dtypes, shape=st.lists(st.integers(0, 4), min_size=0, max_size=4))
def test_roundtrip_property(dt, shape):
    t = (torch.rand(shape) * 10).to(dt)
    v = TensorValue.from_tensor(t)
    stream = io.BytesIO()
    v.write(stream)
    v.write(stream)
    stream.seek(0)
    a = TensorValue.read(stream)
    b = TensorValue.read(stream)
    assert a == v and b == v
    assert torch.equal(a.to_tensor(), t)
    # verbatim record copy (reference copyInternal bug B1 fixed)
    rec, nxt = TensorValue.copy_record(stream.getvalue(), 0)
    assert rec == v.to_bytes() and nxt == len(rec)
    # pickling goes through the framing (B10 fixed)
    assert pickle.loads(pickle.dumps(v)) == v


def test_encode_decode_many():
    vals = [TensorValue.from_tensor(torch.arange(i, dtype=torch.int64)) for i in range(5)]
    assert TensorValue.decode_many(TensorValue.encode_many(vals)) == vals


def test_string_tensor_value():
    s = StringTensor([b"a", b"bcd", b""], shape=(3,))
    v = TensorValue.from_tensor(s)
    assert v.dtype == DataType.STRING
    back = v.to_tensor()
    assert isinstance(back, StringTensor) and back == s
    assert TensorValue.from_bytes(v.to_bytes()).to_tensor() == s


def test_builder_long_is_8_bytes():
    v = TensorValue.builder().data_type(DataType.INT64).shape(3).data([1, 2, 3]).build()
    assert v.nbytes == 24  # reference allocates 4 B per long (B2)
    assert v.to_tensor().tolist() == [1, 2, 3]


def test_dtype_codes():
    assert [get_value(d) for d in (DataType.FLOAT, DataType.DOUBLE, DataType.INT32, DataType.STRING,
                                    DataType.INT64, DataType.BOOL)] == [1, 2, 3, 7, 9, 10]
    assert get_data_type(14) == DataType.BFLOAT16
    assert get_data_type(25) == DataType.FLOAT8_E4M3FN
    assert DataType.FLOAT8_E4M3FN.torch == torch.float8_e4m3fn  # OCP, not fnuz
    with pytest.raises(ValueError):
        get_data_type(14, strict=True)


def test_tensor_name_grammar():
    assert TensorName.parse("foo") == TensorName("foo", 0)
    assert TensorName.parse("foo:3") == TensorName("foo", 3)
    assert str(TensorName.parse("a/b")) == "a/b:0"
    with pytest.raises(ValueError):
        TensorName.parse("a:1:2")


def test_string_packing_native_layout(native):
    elems = [b"x" * 3, b"", b"y" * 200]
    buf = native.string_tensor_pack(elems)
    offs = struct.unpack("<3Q", buf[:24])
    assert offs == (0, 4, 5)
    assert native.string_tensor_unpack(buf, 3) == elems


def test_messages_injection_roundtrip():
    exs = [example(("x", feature(float(v)))) for v in range(4)]
    t = messages_to_tensor(exs)
    assert t.shape == (4,)
    back = tensor_to_messages(t, Example)
    assert [e.features.feature["x"].float_list.value for e in back] == [[0.0], [1.0], [2.0], [3.0]]
    inj = TensorInjections.messages2Tensor(Example)
    assert inj.invert(inj.apply(exs)) == exs
    big = [example(("x", feature(*range(1000)))) for _ in range(20)]  # >10 KB (reference caps at 10,000 B)
    assert len(tensor_to_messages(messages_to_tensor(big), Example)) == 20


def test_arrays_roundtrip_and_tagging():
    a = np.array([1.0, 2.0, 3.0], dtype=np.float32)
    t = array_to_tensor(a)
    tagged_as(t, TypedTensor(1, DataType.FLOAT))
    with pytest.raises(TypeError):
        tagged_as(t, TypedTensor(2, DataType.FLOAT))
    assert np.array_equal(tensor_to_array(t.reshape(1, 3)), a)
    with pytest.raises(ValueError):
        tensor_to_array(torch.zeros(2, 2))


def test_parse_example_dense(native):
    from flink_tensorflow_amd.types.example import FLOAT, encode_float_examples, parse_example_dense

    exs = [example(("x", feature(float(i), float(i) * 2))).encode() for i in range(1000)]
    (x,) = parse_example_dense(exs, [("x", FLOAT, 2, None)])
    assert x.shape == (1000, 2) and x[7].tolist() == [7.0, 14.0]
    (y,) = parse_example_dense(exs, [("missing", FLOAT, 1, [5.0])])
    assert (y == 5.0).all()
    with pytest.raises(ValueError):
        parse_example_dense(exs, [("missing", FLOAT, 1, None)])
    enc = encode_float_examples({"x": np.arange(6, dtype=np.float32).reshape(3, 2)})
    assert [Example.decode(e).features.feature["x"].float_list.value for e in enc] == [[0, 1], [2, 3], [4, 5]]


def test_parse_example_sparse_and_dense_features():
    """TF ``ParseExample`` with ``VarLenFeature`` keys (int64 and bytes) next to a dense
    float key: sparse (indices, values, dense_shape) outputs come first, in TF's order.
    Expected values are written out by hand from the records below (TF is not importable
    here; the layout follows the op's documented output order — parity unpinned)."""
    import numpy as np
    import torch

    from flink_tensorflow_amd.graph.builder import GraphBuilder
    from flink_tensorflow_amd.graph.graph import Graph
    from flink_tensorflow_amd.graph.session import Session
    from flink_tensorflow_amd.proto.messages import TensorShapeProto
    from flink_tensorflow_amd.types.dtypes import DataType
    from flink_tensorflow_amd.types.example import make_example
    from flink_tensorflow_amd.types.tensor import StringTensor

    b = GraphBuilder()
    ser = b.placeholder("ser", "STRING", [None])
    names = b.constant("names", np.asarray([], dtype=object))
    k_ids = b.constant("k_ids", np.asarray(b"ids", dtype=object))
    k_tags = b.constant("k_tags", np.asarray(b"tags", dtype=object))
    k_x = b.constant("k_x", np.asarray(b"x", dtype=object))
    d_x = b.constant("d_x", np.asarray([-1.0], dtype=np.float32))
    b.op("ParseExample", [ser, names, k_ids, k_tags, k_x, d_x], name="parse", Nsparse=2, Ndense=1,
         sparse_types=[DataType.INT64, DataType.STRING], Tdense=[DataType.FLOAT],
         dense_shapes=[TensorShapeProto.of([1])])
    g = Graph.from_graph_def(b.build_graph_def())
    exs = [make_example(ids=[5, 6, 7], tags=[b"a"], x=[1.5]), make_example(tags=[b"b", b"c"]),
           make_example(ids=[9], x=[2.5])]
    feed = StringTensor([e.encode() for e in exs], (3,))
    out = Session(g).run([f"parse:{i}" for i in range(7)], {"ser:0": feed})
    ids_i, tags_i, ids_v, tags_v, ids_s, tags_s, x = out
    assert ids_i.tolist() == [[0, 0], [0, 1], [0, 2], [2, 0]] and ids_v.tolist() == [5, 6, 7, 9]
    assert ids_v.dtype == torch.int64 and ids_s.tolist() == [3, 3]
    assert tags_i.tolist() == [[0, 0], [1, 0], [1, 1]] and tags_v.tolist() == [b"a", b"b", b"c"]
    assert tags_s.tolist() == [3, 2]
    assert x.reshape(-1).tolist() == [1.5, -1.0, 2.5]
