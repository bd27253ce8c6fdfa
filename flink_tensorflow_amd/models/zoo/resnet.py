"""ResNet-50 v1.5 as a frozen TF GraphDef (random-init weights; no network access).

The BASELINE headline config is a ResNet-50 bf16 image-classification stream.  The model
is emitted as a real TF graph (``Conv2D``/``FusedBatchNormV3``/``Relu``/``MaxPool``/``Add``/
``Mean``/``MatMul``/``BiasAdd``/``Softmax``/``TopKV2``) — exactly what a user's frozen
``.pb`` would contain — so it exercises the same path as the reference's GenericModel +
GraphLoader (``EX/inception/InceptionModel.scala:51-62``).  The graph includes the image
normalization front end of ``EX/inception/ImageNormalization.scala:42-77``
(uint8 → Cast → ResizeBilinear → Sub(mean) → Div(std)); the compiler fuses it into one
preprocess kernel and folds every BatchNorm into the conv weights.

Tensor names: ``images`` (uint8 [N,H,W,3]), ``normalized`` (float [N,224,224,3]),
``logits``, ``probs``, ``top_k`` (``top_k:0`` values, ``top_k:1`` indices).
"""
from __future__ import annotations

import numpy as np

from ...graph.builder import GraphBuilder
from ...proto.messages import GraphDef

IMAGENET_MEAN = (123.68, 116.78, 103.94)
IMAGENET_STD = (58.40, 57.12, 57.38)


class _Init:
    def __init__(self, seed):
        self.rng = np.random.default_rng(seed)

    def conv(self, kh, kw, cin, cout):
        std = np.sqrt(2.0 / (kh * kw * cin))
        return (self.rng.standard_normal((kh, kw, cin, cout)) * std).astype(np.float32)

    def bn(self, c, gamma_scale=1.0):
        g = (self.rng.uniform(0.8, 1.2, c) * gamma_scale).astype(np.float32)
        b = (self.rng.standard_normal(c) * 0.05).astype(np.float32)
        m = (self.rng.standard_normal(c) * 0.05).astype(np.float32)
        v = self.rng.uniform(0.8, 1.2, c).astype(np.float32)
        return g, b, m, v


def _conv_bn(gb: GraphBuilder, init: _Init, x, kh, cin, cout, stride, name, relu=True, gamma_scale=1.0,
             residual=None):
    with gb.name_scope(name):
        w = gb.constant("weights", init.conv(kh, kh, cin, cout))
        y = gb.conv2d(x, w, (stride, stride), "SAME", name="Conv2D")
        g, b, m, v = init.bn(cout, gamma_scale)
        y = gb.fused_batch_norm(y, gb.constant("gamma", g), gb.constant("beta", b), gb.constant("moving_mean", m),
                                gb.constant("moving_variance", v), 1.001e-5, name="BatchNorm")
        if residual is not None:
            y = gb.add(y, residual, name="add")
        if relu:
            y = gb.relu(y, name="Relu")
    return y


def resnet50_graph_def(num_classes: int = 1000, seed: int = 0, image_hw: tuple[int, int] | None = None,
                       out_hw: tuple[int, int] = (224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD,
                       top_k: int = 5, depth: int = 50) -> GraphDef:
    blocks = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3], 26: [2, 2, 2, 2]}[depth]
    gb = GraphBuilder()
    init = _Init(seed)
    shape = [None, image_hw[0], image_hw[1], 3] if image_hw else [None, None, None, 3]
    images = gb.placeholder("images", "UINT8", shape)
    x = gb.cast(images, "FLOAT", name="Cast")
    x = gb.resize_bilinear(x, gb.constant("size", np.asarray(out_hw, dtype=np.int32)), name="ResizeBilinear")
    x = gb.sub(x, gb.constant("mean", np.asarray(mean, dtype=np.float32)), name="Sub")
    x = gb.div(x, gb.constant("std", np.asarray(std, dtype=np.float32)), name="normalized")
    x = _conv_bn(gb, init, x, 7, 3, 64, 2, "conv1")
    x = gb.max_pool(x, (3, 3), (2, 2), "SAME", name="pool1")
    cin = 64
    for stage, (n, width) in enumerate(zip(blocks, [64, 128, 256, 512])):
        for i in range(n):
            stride = 2 if (i == 0 and stage > 0) else 1
            cout = width * 4
            name = f"block{stage + 1}/unit{i + 1}"
            if i == 0:
                shortcut = _conv_bn(gb, init, x, 1, cin, cout, stride, name + "/shortcut", relu=False)
            else:
                shortcut = x
            y = _conv_bn(gb, init, x, 1, cin, width, 1, name + "/conv1")
            y = _conv_bn(gb, init, y, 3, width, width, stride, name + "/conv2")  # v1.5: stride on the 3x3
            x = _conv_bn(gb, init, y, 1, width, cout, 1, name + "/conv3", gamma_scale=0.3, residual=shortcut)
            cin = cout
    x = gb.mean(x, [1, 2], name="avg_pool")
    w = gb.constant("fc/weights", (init.rng.standard_normal((2048, num_classes)) * np.sqrt(1.0 / 2048)).astype(np.float32))
    b = gb.constant("fc/biases", np.zeros(num_classes, dtype=np.float32))
    logits = gb.bias_add(gb.matmul(x, w, name="fc/MatMul"), b, name="logits")
    probs = gb.softmax(logits, name="probs")
    gb.top_k(probs, top_k, name="top_k")
    return gb.build_graph_def()


def resnet50_flops_per_image(hw=224) -> float:
    """Forward FLOPs (2·MAC) of ResNet-50 v1.5 at hw×hw (≈8.2 GFLOP at 224)."""
    return 4.09e9 * 2 * (hw / 224) ** 2


def export_resnet50_saved_model(export_dir: str, image_hw: tuple[int, int] | None = None, seed: int = 0,
                                top_k: int = 5, depth: int = 50, num_classes: int = 1000) -> str:
    """ResNet-50 v1.5 (random init) as a real TF 1.x SavedModel: weights are variables in
    ``variables/`` and the ``serving_default`` predict signature maps ``images`` (uint8
    NHWC) to ``probabilities`` / ``scores`` / ``classes`` (top-k)."""
    from ...proto.messages import SignatureDef
    from ..export import graph_def_to_saved_model, tensor_info

    gd = resnet50_graph_def(num_classes=num_classes, seed=seed, image_hw=image_hw, top_k=top_k, depth=depth)
    hw = list(image_hw) if image_hw else [-1, -1]
    sig = SignatureDef(inputs={"images": tensor_info("images:0", "UINT8", [-1, *hw, 3])},
                       outputs={"probabilities": tensor_info("probs:0", "FLOAT", [-1, num_classes]),
                                "scores": tensor_info("top_k:0", "FLOAT", [-1, top_k]),
                                "classes": tensor_info("top_k:1", "INT32", [-1, top_k])},
                       method_name="tensorflow/serving/predict")
    return graph_def_to_saved_model(export_dir, gd, {"serving_default": sig})
