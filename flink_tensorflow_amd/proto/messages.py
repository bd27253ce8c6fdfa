"""TensorFlow 1.x protobuf messages used by SavedModels, GraphDefs, checkpoints and tf.Example.

Field numbers follow the public ``tensorflow/core/framework/*.proto``,
``tensorflow/core/protobuf/{meta_graph,saved_model,saver,tensor_bundle}.proto`` and
``tensorflow/core/example/{example,feature}.proto`` definitions.  These are the message
types the reference registers with Kryo (``LIB/util/RegistrationUtils.java:23-85``) and
that ``R/models/half_plus_two/saved_model.pb`` contains.
"""
from __future__ import annotations

from .wire import F, Message

# ----------------------------------------------------------------------------- framework


class VersionDef(Message):
    FIELDS = [F(1, "producer", "int32"), F(2, "min_consumer", "int32"),
              F(3, "bad_consumers", "int32", repeated=True)]


class TensorShapeDim(Message):
    FIELDS = [F(1, "size", "int64"), F(2, "name", "string")]


class TensorShapeProto(Message):
    FIELDS = [F(2, "dim", "message", repeated=True, msg=TensorShapeDim), F(3, "unknown_rank", "bool")]

    @classmethod
    def of(cls, dims) -> "TensorShapeProto":
        if dims is None:
            return cls(unknown_rank=True)
        return cls(dim=[TensorShapeDim(size=int(d) if d is not None else -1) for d in dims])

    def as_list(self):
        if self.unknown_rank:
            return None
        return [d.size for d in self.dim]


class ResourceHandleProto(Message):
    FIELDS = [F(1, "device", "string"), F(2, "container", "string"), F(3, "name", "string"),
              F(4, "hash_code", "uint64"), F(5, "maybe_type_name", "string")]


class TensorProto(Message):
    FIELDS = [
        F(1, "dtype", "enum"),
        F(2, "tensor_shape", "message", msg=TensorShapeProto),
        F(3, "version_number", "int32"),
        F(4, "tensor_content", "bytes"),
        F(5, "float_val", "float", repeated=True),
        F(6, "double_val", "double", repeated=True),
        F(7, "int_val", "int32", repeated=True),
        F(8, "string_val", "bytes", repeated=True),
        F(9, "scomplex_val", "float", repeated=True),
        F(10, "int64_val", "int64", repeated=True),
        F(11, "bool_val", "bool", repeated=True),
        F(12, "dcomplex_val", "double", repeated=True),
        F(13, "half_val", "int32", repeated=True),
        F(14, "resource_handle_val", "message", repeated=True, msg=ResourceHandleProto),
        F(16, "uint32_val", "uint32", repeated=True),
        F(17, "uint64_val", "uint64", repeated=True),
    ]


class NameAttrList(Message):
    FIELDS = [F(1, "name", "string"), F(2, "attr", "map", msg=lambda: AttrValue)]


class AttrListValue(Message):
    FIELDS = [
        F(2, "s", "bytes", repeated=True),
        F(3, "i", "int64", repeated=True),
        F(4, "f", "float", repeated=True),
        F(5, "b", "bool", repeated=True),
        F(6, "type", "enum", repeated=True),
        F(7, "shape", "message", repeated=True, msg=TensorShapeProto),
        F(8, "tensor", "message", repeated=True, msg=TensorProto),
        F(9, "func", "message", repeated=True, msg=NameAttrList),
    ]


class AttrValue(Message):
    """``oneof value { list=1 s=2 i=3 f=4 b=5 type=6 shape=7 tensor=8 placeholder=9 func=10 }``.

    proto3 oneof members are emitted even at default values; ``which`` records the member
    so that e.g. ``b=False`` or ``i=0`` survive a round trip."""

    FIELDS = [
        F(1, "list", "message", msg=AttrListValue),
        F(2, "s", "bytes"),
        F(3, "i", "int64"),
        F(4, "f", "float"),
        F(5, "b", "bool"),
        F(6, "type", "enum"),
        F(7, "shape", "message", msg=TensorShapeProto),
        F(8, "tensor", "message", msg=TensorProto),
        F(9, "placeholder", "string"),
        F(10, "func", "message", msg=NameAttrList),
    ]

    @classmethod
    def decode(cls, buf):
        from .wire import scan

        self = super().decode(buf)
        nums = [n for n, _, _ in scan(bytes(buf))]
        self.which = cls._by_num[nums[-1]].name if nums and nums[-1] in cls._by_num else None
        return self

    def __init__(self, **kw):
        super().__init__(**kw)
        self.which = next(iter(kw)) if len(kw) == 1 else None

    def encode(self) -> bytes:
        from .wire import _encode_scalar_payload, _key, encode_varint

        w = self.which
        if w is None:
            return super().encode()
        f = self._by_name[w]
        v = getattr(self, w)
        if f.kind == "message":
            b = (v or f.msg_cls()()).encode()
            return _key(f.number, 2) + encode_varint(len(b)) + b
        wt, p = _encode_scalar_payload(f.kind, v)
        return _key(f.number, wt) + p

    def value(self):
        """The python value of the set oneof member."""
        if self.which is None:
            return None
        if self.which == "list":
            lv = self.list or AttrListValue()
            for name in ("s", "i", "f", "b", "type", "shape", "tensor", "func"):
                if getattr(lv, name):
                    return list(getattr(lv, name))
            return []
        return getattr(self, self.which)


class NodeDef(Message):
    FIELDS = [F(1, "name", "string"), F(2, "op", "string"), F(3, "input", "string", repeated=True),
              F(4, "device", "string"), F(5, "attr", "map", msg=AttrValue)]


class OpDefRaw(Message):
    """OpDef kept mostly opaque (only the name is interpreted)."""

    FIELDS = [F(1, "name", "string")]


class OpList(Message):
    FIELDS = [F(1, "op", "message", repeated=True, msg=OpDefRaw)]


class ArgDef(Message):
    """``OpDef.ArgDef``: one input / output argument of an op or function signature."""

    FIELDS = [F(1, "name", "string"), F(2, "description", "string"), F(3, "type", "enum"),
              F(4, "type_attr", "string"), F(5, "number_attr", "string"), F(6, "type_list_attr", "string"),
              F(16, "is_ref", "bool")]


class AttrDef(Message):
    FIELDS = [F(1, "name", "string"), F(2, "type", "string"), F(3, "default_value", "message", msg=AttrValue)]


class OpDef(Message):
    """A function signature (``FunctionDef.signature``)."""

    FIELDS = [F(1, "name", "string"), F(2, "input_arg", "message", repeated=True, msg=ArgDef),
              F(3, "output_arg", "message", repeated=True, msg=ArgDef),
              F(4, "attr", "message", repeated=True, msg=AttrDef), F(5, "summary", "string"),
              F(6, "description", "string"), F(16, "is_aggregate", "bool"), F(17, "is_stateful", "bool"),
              F(18, "is_commutative", "bool"), F(19, "allows_uninitialized_input", "bool"),
              F(20, "control_output", "string", repeated=True)]  # op_def.proto field numbers


class FunctionDef(Message):
    """``tensorflow/core/framework/function.proto``: a function body.  Inside it, inputs
    name the signature's arguments (``"x"``) or node outputs as ``"node:out_arg:index"``."""

    FIELDS = [F(1, "signature", "message", msg=OpDef), F(3, "node_def", "message", repeated=True, msg=NodeDef),
              F(4, "ret", "map", value_kind="string"), F(5, "attr", "map", msg=AttrValue),
              F(6, "control_ret", "map", value_kind="string")]


class GradientDef(Message):
    FIELDS = [F(1, "function_name", "string"), F(2, "gradient_func", "string")]


class FunctionDefLibrary(Message):
    FIELDS = [F(1, "function", "message", repeated=True, msg=FunctionDef),
              F(2, "gradient", "message", repeated=True, msg=GradientDef)]


class GraphDef(Message):
    FIELDS = [F(1, "node", "message", repeated=True, msg=NodeDef), F(2, "library", "message", msg=FunctionDefLibrary),
              F(3, "version", "int32"), F(4, "versions", "message", msg=VersionDef)]


# ----------------------------------------------------------------------------- meta graph


class AnyProto(Message):
    FIELDS = [F(1, "type_url", "string"), F(2, "value", "bytes")]


class MetaInfoDef(Message):
    FIELDS = [
        F(1, "meta_graph_version", "string"),
        F(2, "stripped_op_list", "message", msg=OpList),
        F(3, "any_info", "message", msg=AnyProto),
        F(4, "tags", "string", repeated=True),
        F(5, "tensorflow_version", "string"),
        F(6, "tensorflow_git_version", "string"),
        F(7, "stripped_default_attrs", "bool"),
    ]


class NodeList(Message):
    FIELDS = [F(1, "value", "string", repeated=True)]


class BytesListC(Message):
    FIELDS = [F(1, "value", "bytes", repeated=True)]


class Int64ListC(Message):
    FIELDS = [F(1, "value", "int64", repeated=True)]


class FloatListC(Message):
    FIELDS = [F(1, "value", "float", repeated=True)]


class AnyListC(Message):
    FIELDS = [F(1, "value", "message", repeated=True, msg=AnyProto)]


class CollectionDef(Message):
    FIELDS = [F(1, "node_list", "message", msg=NodeList), F(2, "bytes_list", "message", msg=BytesListC),
              F(3, "int64_list", "message", msg=Int64ListC), F(4, "float_list", "message", msg=FloatListC),
              F(5, "any_list", "message", msg=AnyListC)]


class TensorInfo(Message):
    FIELDS = [F(1, "name", "string"), F(2, "dtype", "enum"), F(3, "tensor_shape", "message", msg=TensorShapeProto)]


class SignatureDef(Message):
    FIELDS = [F(1, "inputs", "map", msg=TensorInfo), F(2, "outputs", "map", msg=TensorInfo),
              F(3, "method_name", "string")]


class SaverDef(Message):
    LEGACY, V1, V2 = 0, 1, 2
    FIELDS = [
        F(1, "filename_tensor_name", "string"),
        F(2, "save_tensor_name", "string"),
        F(3, "restore_op_name", "string"),
        F(4, "max_to_keep", "int32"),
        F(5, "sharded", "bool"),
        F(6, "keep_checkpoint_every_n_hours", "float"),
        F(7, "version", "enum"),
    ]


class AssetFileDef(Message):
    FIELDS = [F(1, "tensor_info", "message", msg=TensorInfo), F(2, "filename", "string")]


class MetaGraphDef(Message):
    FIELDS = [
        F(1, "meta_info_def", "message", msg=MetaInfoDef),
        F(2, "graph_def", "message", msg=GraphDef),
        F(3, "saver_def", "message", msg=SaverDef),
        F(4, "collection_def", "map", msg=CollectionDef),
        F(5, "signature_def", "map", msg=SignatureDef),
        F(6, "asset_file_def", "message", repeated=True, msg=AssetFileDef),
    ]


class SavedModel(Message):
    FIELDS = [F(1, "saved_model_schema_version", "int64"),
              F(2, "meta_graphs", "message", repeated=True, msg=MetaGraphDef)]


# ----------------------------------------------------------------------------- tf.Example


class BytesList(Message):
    FIELDS = [F(1, "value", "bytes", repeated=True)]


class FloatList(Message):
    FIELDS = [F(1, "value", "float", repeated=True)]


class Int64List(Message):
    FIELDS = [F(1, "value", "int64", repeated=True)]


class Feature(Message):
    FIELDS = [F(1, "bytes_list", "message", msg=BytesList), F(2, "float_list", "message", msg=FloatList),
              F(3, "int64_list", "message", msg=Int64List)]


class Features(Message):
    FIELDS = [F(1, "feature", "map", msg=Feature)]


class Example(Message):
    FIELDS = [F(1, "features", "message", msg=Features)]


class FeatureList(Message):
    FIELDS = [F(1, "feature", "message", repeated=True, msg=Feature)]


class FeatureLists(Message):
    FIELDS = [F(1, "feature_list", "map", msg=FeatureList)]


class SequenceExample(Message):
    FIELDS = [F(1, "context", "message", msg=Features), F(2, "feature_lists", "message", msg=FeatureLists)]


# ----------------------------------------------------------------------------- tensor bundle


class TensorSliceExtent(Message):
    FIELDS = [F(1, "start", "int64"), F(2, "length", "int64")]


class TensorSliceProto(Message):
    FIELDS = [F(1, "extent", "message", repeated=True, msg=TensorSliceExtent)]


class BundleHeaderProto(Message):
    LITTLE, BIG = 0, 1
    FIELDS = [F(1, "num_shards", "int32"), F(2, "endianness", "enum"), F(3, "version", "message", msg=VersionDef)]


class BundleEntryProto(Message):
    FIELDS = [
        F(1, "dtype", "enum"),
        F(2, "shape", "message", msg=TensorShapeProto),
        F(3, "shard_id", "int32"),
        F(4, "offset", "int64"),
        F(5, "size", "int64"),
        F(6, "crc32c", "fixed32"),
        F(7, "slices", "message", repeated=True, msg=TensorSliceProto),
    ]


# ----------------------------------------------------------------------------- run metadata


class NodeExecStats(Message):
    FIELDS = [F(1, "node_name", "string"), F(2, "all_start_micros", "int64"), F(3, "op_start_rel_micros", "int64"),
              F(4, "op_end_rel_micros", "int64"), F(5, "all_end_rel_micros", "int64"),
              F(8, "timeline_label", "string")]


class DeviceStepStats(Message):
    FIELDS = [F(1, "device", "string"), F(2, "node_stats", "message", repeated=True, msg=NodeExecStats)]


class StepStats(Message):
    FIELDS = [F(1, "dev_stats", "message", repeated=True, msg=DeviceStepStats)]


class RunMetadata(Message):
    FIELDS = [F(1, "step_stats", "message", msg=StepStats)]


REGISTERED_TYPES = [
    Example, SequenceExample, Feature, Features, FeatureList, FeatureLists, BytesList, FloatList, Int64List,
    GraphDef, NodeDef, AttrValue, TensorProto, TensorShapeProto, MetaGraphDef, SignatureDef, TensorInfo,
    SaverDef, SavedModel, CollectionDef, BundleHeaderProto, BundleEntryProto, RunMetadata, StepStats,
    NodeExecStats, DeviceStepStats, VersionDef,
]
