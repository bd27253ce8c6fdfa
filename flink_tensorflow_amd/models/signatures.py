"""Standard TF-Serving signature methods.

``RegressionMethod`` mirrors ``LIB/ml/signatures/RegressionMethod.scala:18-36`` (input a
STRING tensor of serialized ``tf.Example``s, output ``outputs`` float [N,1]).
``PredictMethod`` and ``ClassificationMethod`` are added: the reference defines their
constants (``SignatureConstants.java``) and the half_plus_two fixture carries
``serving_default`` (predict) and ``classify_x_to_y`` signatures, but never implements them.
"""
from __future__ import annotations

from typing import Mapping

from ..types.codecs import messages_to_tensor
from ..types.dtypes import DataType
from ..types.names import TypedTensor, tagged_as
from .core import GraphMethod
from .savedmodel import SignatureConstants as SC

ExampleTensor = TypedTensor(None, DataType.STRING)
PredictionTensor = TypedTensor(2, DataType.FLOAT)


def _examples(value):
    if isinstance(value, (list, tuple)) and value and hasattr(value[0], "SerializeToString"):
        return messages_to_tensor(value)
    return value


class RegressionMethod(GraphMethod):
    name = SC.REGRESS_METHOD_NAME

    def inputs(self, value) -> Mapping:
        return {SC.REGRESS_INPUTS: _examples(value)}

    def outputs(self, tensors):
        return tagged_as(tensors[SC.REGRESS_OUTPUTS], PredictionTensor)


class ClassificationMethod(GraphMethod):
    """Outputs ``(classes or None, scores or None)``."""

    name = SC.CLASSIFY_METHOD_NAME

    def inputs(self, value) -> Mapping:
        return {SC.CLASSIFY_INPUTS: _examples(value)}

    def outputs(self, tensors):
        return tensors.get(SC.CLASSIFY_OUTPUT_CLASSES), tensors.get(SC.CLASSIFY_OUTPUT_SCORES)


class PredictMethod(GraphMethod):
    """Generic predict: ``inputs`` is a dict keyed like the signature's inputs; returns
    the full output dict."""

    name = SC.PREDICT_METHOD_NAME

    def inputs(self, value) -> Mapping:
        if not isinstance(value, Mapping):
            return {SC.PREDICT_INPUTS: value}
        return value

    def outputs(self, tensors):
        return dict(tensors)


class LambdaMethod(GraphMethod):
    """Ad-hoc method from two callables (handy for GenericModel signatures)."""

    def __init__(self, name: str, inputs, outputs):
        self.name = name
        self._in = inputs
        self._out = outputs

    def inputs(self, value):
        return self._in(value)

    def outputs(self, tensors):
        return self._out(tensors)
