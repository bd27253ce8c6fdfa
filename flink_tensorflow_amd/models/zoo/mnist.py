"""MNIST MLP SavedModel — the BASELINE "CPU plumbing" config.

``export_mnist_mlp(dir)`` writes a real TF 1.x SavedModel (``serve`` tag) with
signatures ``serving_default`` (predict: ``images`` float [N,784] → ``scores`` [N,10]),
``classify_images`` (classify: ``classes`` int64 + ``scores``) and ``regress_examples``
(regress over serialized ``tf.Example{"pixels": float[784]}`` → ``outputs`` = P(digit 0)),
random-init weights (no dataset download).  ``MnistModel`` is the ``TensorFlowModel``.
"""
from __future__ import annotations

import numpy as np

from ...graph.builder import GraphBuilder
from ...proto.messages import SignatureDef, TensorShapeProto
from ..export import export_saved_model, tensor_info
from ..savedmodel import SignatureConstants as SC
from ..savedmodel import TensorFlowModel


def export_mnist_mlp(export_dir: str, hidden: int = 128, seed: int = 0) -> str:
    rng = np.random.default_rng(seed)
    b = GraphBuilder()
    w1v = (rng.standard_normal((784, hidden)) * np.sqrt(2 / 784)).astype(np.float32)
    b1v = np.zeros(hidden, np.float32)
    w2v = (rng.standard_normal((hidden, 10)) * np.sqrt(1 / hidden)).astype(np.float32)
    b2v = np.zeros(10, np.float32)
    w1 = b.variable_with_init("dense/kernel", w1v)
    b1 = b.variable_with_init("dense/bias", b1v)
    w2 = b.variable_with_init("logits/kernel", w2v)
    b2 = b.variable_with_init("logits/bias", b2v)
    images = b.placeholder("images", "FLOAT", [None, 784])
    # regress path: serialized tf.Examples -> pixels
    ex = b.placeholder("tf_example", "STRING", [None])
    names = b.constant("ParseExample/names", np.asarray([], dtype=object))
    key = b.constant("ParseExample/dense_keys_0", np.asarray(b"pixels", dtype=object))
    dflt = b.constant("ParseExample/default", np.zeros(0, np.float32))
    pixels = b.op("ParseExample", [ex, names, key, dflt], name="ParseExample", Nsparse=0, Ndense=1,
                  Tdense=[__import__("flink_tensorflow_amd").types.DataType.FLOAT],
                  dense_shapes=[TensorShapeProto.of([784])], sparse_types=[])

    def mlp(x, scope):
        with b.name_scope(scope):
            h = b.relu(b.bias_add(b.matmul(x, w1), b1))
            logits = b.bias_add(b.matmul(h, w2), b2, name="logits")
            return logits, b.softmax(logits, name="scores")

    logits, scores = mlp(images, "predict")
    _, ex_scores = mlp(pixels, "regress")
    p0 = b.op("Slice", [ex_scores, b.constant("p0/begin", np.asarray([0, 0], np.int32)),
                        b.constant("p0/size", np.asarray([-1, 1], np.int32))], name="p0")
    classes = b.op("ArgMax", [scores, b.constant("argmax/dim", np.int32(1))], name="classes",
                   output_type=__import__("flink_tensorflow_amd").types.DataType.INT64)
    sigs = {
        SC.DEFAULT_SERVING_SIGNATURE_DEF_KEY: SignatureDef(
            inputs={"images": tensor_info(images, "FLOAT", [-1, 784])},
            outputs={"scores": tensor_info(scores, "FLOAT", [-1, 10]), "logits": tensor_info(logits, "FLOAT", [-1, 10])},
            method_name=SC.PREDICT_METHOD_NAME),
        "classify_images": SignatureDef(
            inputs={SC.CLASSIFY_INPUTS: tensor_info(images, "FLOAT", [-1, 784])},
            outputs={SC.CLASSIFY_OUTPUT_CLASSES: tensor_info(classes, "INT64", [-1]),
                     SC.CLASSIFY_OUTPUT_SCORES: tensor_info(scores, "FLOAT", [-1, 10])},
            method_name=SC.CLASSIFY_METHOD_NAME),
        "regress_examples": SignatureDef(
            inputs={SC.REGRESS_INPUTS: tensor_info(ex, "STRING", [-1])},
            outputs={SC.REGRESS_OUTPUTS: tensor_info(p0, "FLOAT", [-1, 1])},
            method_name=SC.REGRESS_METHOD_NAME),
    }
    return export_saved_model(export_dir, b, {"dense/kernel": w1v, "dense/bias": b1v, "logits/kernel": w2v,
                                              "logits/bias": b2v}, sigs)


class MnistModel(TensorFlowModel):
    def __init__(self, path: str, device="cpu"):
        super().__init__(device)
        self._loader = TensorFlowModel.load(path, "serve")

    @property
    def loader(self):
        return self._loader

    def predict(self, images):
        from ..signatures import PredictMethod

        return self.function(SC.DEFAULT_SERVING_SIGNATURE_DEF_KEY, PredictMethod()).apply({"images": images})

    def classify(self, images):
        from ..signatures import ClassificationMethod

        return self.function("classify_images", ClassificationMethod()).apply(images)
