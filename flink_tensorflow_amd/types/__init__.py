"""L3 tensor types and conversions (SURVEY §2.1, T1–T11)."""
from .codecs import (Injection, TensorInjections, array_to_tensor, bytes_to_tensor, message_to_tensor,
                     messages_to_tensor, scalar_to_tensor, tensor_to_array, tensor_to_bytes, tensor_to_message,
                     tensor_to_messages, tensor_to_scalar, to_graph_tensor, to_value, value_to_tensor)
from .dtypes import DataType, get_data_type, get_value
from .example import example, feature, make_example, parse_example_dense
from .names import ANY_RANK, Rank, TensorName, TypedTensor, TypeTag, tagged_as, tagged_with
from .tensor import StringTensor, as_tensor, dtype_of, shape_of
from .tensor_value import TensorValue, TensorValueBuilder, VersionMismatchException

__all__ = [
    "DataType", "get_data_type", "get_value", "TensorValue", "TensorValueBuilder", "VersionMismatchException",
    "StringTensor", "as_tensor", "dtype_of", "shape_of", "TensorName", "Rank", "TypedTensor", "TypeTag",
    "tagged_as", "tagged_with", "ANY_RANK", "Injection", "TensorInjections", "scalar_to_tensor",
    "tensor_to_scalar", "array_to_tensor", "tensor_to_array", "bytes_to_tensor", "tensor_to_bytes",
    "message_to_tensor", "tensor_to_message", "messages_to_tensor", "tensor_to_messages", "value_to_tensor",
    "to_value", "to_graph_tensor", "example", "feature", "make_example", "parse_example_dense",
]
