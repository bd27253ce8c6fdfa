"""Inception-v3 (299×299) as a frozen TF GraphDef with random-init weights — the model of
BASELINE config 5 ("Inception-v3 fp8 weights (CDNA4 fp8 MFMA) with dynamic per-operator
batching").  The reference's Inception example labels images with a frozen Inception
graph (``EX/inception/InceptionModel.scala:51-62``); this builder emits the v3 topology
(stem, 3× Mixed_5 35×35, Mixed_6a reduction, 4× Mixed_6 17×17 with factorised 1×7/7×1
convs, Mixed_7a reduction, 2× Mixed_7 8×8 with split 1×3/3×1 branches, global average
pool, 1001-way classifier) with every conv as ``Conv2D → FusedBatchNormV3 → Relu``.

The Mixed_7 blocks' nested concats (``concat([1×3, 3×1])`` inside the block concat) are
emitted flat — the same tensor — so every branch writes straight into one buffer.

Tensor names: ``images`` (uint8 [N,H,W,3]), ``normalized``, ``logits``, ``probs``,
``top_k`` (``top_k:0`` values, ``top_k:1`` indices).
"""
from __future__ import annotations

import numpy as np

from ...graph.builder import GraphBuilder
from ...proto.messages import GraphDef
from .resnet import _Init


def _conv(gb: GraphBuilder, init: _Init, x, cin, cout, k, stride=1, padding="SAME", name="conv"):
    kh, kw = (k, k) if isinstance(k, int) else k
    with gb.name_scope(name):
        w = gb.constant("weights", init.conv(kh, kw, cin, cout) if kh == kw else _rect(init, kh, kw, cin, cout))
        y = gb.conv2d(x, w, (stride, stride), padding, name="Conv2D")
        g, b, m, v = init.bn(cout)
        y = gb.fused_batch_norm(y, gb.constant("gamma", g), gb.constant("beta", b), gb.constant("moving_mean", m),
                                gb.constant("moving_variance", v), 1e-3, name="BatchNorm")
        return gb.relu(y, name="Relu")


def _rect(init: _Init, kh, kw, cin, cout):
    std = np.sqrt(2.0 / (kh * kw * cin))
    return (init.rng.standard_normal((kh, kw, cin, cout)) * std).astype(np.float32)


def _block_a(gb, init, x, cin, pool_ch, name):
    """Mixed_5b/5c/5d (35×35): 1×1 | 1×1→5×5 | 1×1→3×3→3×3 | avgpool→1×1."""
    with gb.name_scope(name):
        b0 = _conv(gb, init, x, cin, 64, 1, name="Branch_0/Conv2d_0a_1x1")
        b1 = _conv(gb, init, x, cin, 48, 1, name="Branch_1/Conv2d_0a_1x1")
        b1 = _conv(gb, init, b1, 48, 64, 5, name="Branch_1/Conv2d_0b_5x5")
        b2 = _conv(gb, init, x, cin, 64, 1, name="Branch_2/Conv2d_0a_1x1")
        b2 = _conv(gb, init, b2, 64, 96, 3, name="Branch_2/Conv2d_0b_3x3")
        b2 = _conv(gb, init, b2, 96, 96, 3, name="Branch_2/Conv2d_0c_3x3")
        b3 = gb.avg_pool(x, (3, 3), (1, 1), "SAME", name="Branch_3/AvgPool_0a_3x3")
        b3 = _conv(gb, init, b3, cin, pool_ch, 1, name="Branch_3/Conv2d_0b_1x1")
        return gb.concat([b0, b1, b2, b3], 3, name="concat"), 64 + 64 + 96 + pool_ch


def _block_b(gb, init, x, cin, c7, name):
    """Mixed_6b..6e (17×17): factorised 7×7 convolutions."""
    with gb.name_scope(name):
        b0 = _conv(gb, init, x, cin, 192, 1, name="Branch_0/Conv2d_0a_1x1")
        b1 = _conv(gb, init, x, cin, c7, 1, name="Branch_1/Conv2d_0a_1x1")
        b1 = _conv(gb, init, b1, c7, c7, (1, 7), name="Branch_1/Conv2d_0b_1x7")
        b1 = _conv(gb, init, b1, c7, 192, (7, 1), name="Branch_1/Conv2d_0c_7x1")
        b2 = _conv(gb, init, x, cin, c7, 1, name="Branch_2/Conv2d_0a_1x1")
        b2 = _conv(gb, init, b2, c7, c7, (7, 1), name="Branch_2/Conv2d_0b_7x1")
        b2 = _conv(gb, init, b2, c7, c7, (1, 7), name="Branch_2/Conv2d_0c_1x7")
        b2 = _conv(gb, init, b2, c7, c7, (7, 1), name="Branch_2/Conv2d_0d_7x1")
        b2 = _conv(gb, init, b2, c7, 192, (1, 7), name="Branch_2/Conv2d_0e_1x7")
        b3 = gb.avg_pool(x, (3, 3), (1, 1), "SAME", name="Branch_3/AvgPool_0a_3x3")
        b3 = _conv(gb, init, b3, cin, 192, 1, name="Branch_3/Conv2d_0b_1x1")
        return gb.concat([b0, b1, b2, b3], 3, name="concat"), 768


def _block_c(gb, init, x, cin, name):
    """Mixed_7b/7c (8×8): split 1×3 / 3×1 branches (flattened concat)."""
    with gb.name_scope(name):
        b0 = _conv(gb, init, x, cin, 320, 1, name="Branch_0/Conv2d_0a_1x1")
        b1 = _conv(gb, init, x, cin, 384, 1, name="Branch_1/Conv2d_0a_1x1")
        b1a = _conv(gb, init, b1, 384, 384, (1, 3), name="Branch_1/Conv2d_0b_1x3")
        b1b = _conv(gb, init, b1, 384, 384, (3, 1), name="Branch_1/Conv2d_0b_3x1")
        b2 = _conv(gb, init, x, cin, 448, 1, name="Branch_2/Conv2d_0a_1x1")
        b2 = _conv(gb, init, b2, 448, 384, 3, name="Branch_2/Conv2d_0b_3x3")
        b2a = _conv(gb, init, b2, 384, 384, (1, 3), name="Branch_2/Conv2d_0c_1x3")
        b2b = _conv(gb, init, b2, 384, 384, (3, 1), name="Branch_2/Conv2d_0d_3x1")
        b3 = gb.avg_pool(x, (3, 3), (1, 1), "SAME", name="Branch_3/AvgPool_0a_3x3")
        b3 = _conv(gb, init, b3, cin, 192, 1, name="Branch_3/Conv2d_0b_1x1")
        return gb.concat([b0, b1a, b1b, b2a, b2b, b3], 3, name="concat"), 2048


def inception_v3_graph_def(num_classes: int = 1001, seed: int = 0, image_hw: tuple[int, int] | None = None,
                           out_hw: tuple[int, int] = (299, 299), top_k: int = 5) -> GraphDef:
    gb = GraphBuilder()
    init = _Init(seed)
    shape = [None, image_hw[0], image_hw[1], 3] if image_hw else [None, None, None, 3]
    images = gb.placeholder("images", "UINT8", shape)
    x = gb.cast(images, "FLOAT", name="Cast")
    x = gb.resize_bilinear(x, gb.constant("size", np.asarray(out_hw, dtype=np.int32)), name="ResizeBilinear")
    x = gb.sub(x, gb.constant("mean", np.asarray([127.5] * 3, dtype=np.float32)), name="Sub")
    x = gb.div(x, gb.constant("std", np.asarray([127.5] * 3, dtype=np.float32)), name="normalized")
    with gb.name_scope("InceptionV3"):
        x = _conv(gb, init, x, 3, 32, 3, 2, "VALID", "Conv2d_1a_3x3")
        x = _conv(gb, init, x, 32, 32, 3, 1, "VALID", "Conv2d_2a_3x3")
        x = _conv(gb, init, x, 32, 64, 3, 1, "SAME", "Conv2d_2b_3x3")
        x = gb.max_pool(x, (3, 3), (2, 2), "VALID", name="MaxPool_3a_3x3")
        x = _conv(gb, init, x, 64, 80, 1, 1, "VALID", "Conv2d_3b_1x1")
        x = _conv(gb, init, x, 80, 192, 3, 1, "VALID", "Conv2d_4a_3x3")
        x = gb.max_pool(x, (3, 3), (2, 2), "VALID", name="MaxPool_5a_3x3")
        x, c = _block_a(gb, init, x, 192, 32, "Mixed_5b")
        x, c = _block_a(gb, init, x, c, 64, "Mixed_5c")
        x, c = _block_a(gb, init, x, c, 64, "Mixed_5d")
        with gb.name_scope("Mixed_6a"):
            b0 = _conv(gb, init, x, c, 384, 3, 2, "VALID", "Branch_0/Conv2d_1a_1x1")
            b1 = _conv(gb, init, x, c, 64, 1, name="Branch_1/Conv2d_0a_1x1")
            b1 = _conv(gb, init, b1, 64, 96, 3, name="Branch_1/Conv2d_0b_3x3")
            b1 = _conv(gb, init, b1, 96, 96, 3, 2, "VALID", "Branch_1/Conv2d_1a_1x1")
            b2 = gb.max_pool(x, (3, 3), (2, 2), "VALID", name="Branch_2/MaxPool_1a_3x3")
            x, c = gb.concat([b0, b1, b2], 3, name="concat"), 384 + 96 + c
        for name, c7 in (("Mixed_6b", 128), ("Mixed_6c", 160), ("Mixed_6d", 160), ("Mixed_6e", 192)):
            x, c = _block_b(gb, init, x, c, c7, name)
        with gb.name_scope("Mixed_7a"):
            b0 = _conv(gb, init, x, c, 192, 1, name="Branch_0/Conv2d_0a_1x1")
            b0 = _conv(gb, init, b0, 192, 320, 3, 2, "VALID", "Branch_0/Conv2d_1a_3x3")
            b1 = _conv(gb, init, x, c, 192, 1, name="Branch_1/Conv2d_0a_1x1")
            b1 = _conv(gb, init, b1, 192, 192, (1, 7), name="Branch_1/Conv2d_0b_1x7")
            b1 = _conv(gb, init, b1, 192, 192, (7, 1), name="Branch_1/Conv2d_0c_7x1")
            b1 = _conv(gb, init, b1, 192, 192, 3, 2, "VALID", "Branch_1/Conv2d_1a_3x3")
            b2 = gb.max_pool(x, (3, 3), (2, 2), "VALID", name="Branch_2/MaxPool_1a_3x3")
            x, c = gb.concat([b0, b1, b2], 3, name="concat"), 320 + 192 + c
        x, c = _block_c(gb, init, x, c, "Mixed_7b")
        x, c = _block_c(gb, init, x, c, "Mixed_7c")
        x = gb.mean(x, [1, 2], name="AvgPool")
    w = gb.constant("Logits/weights", (init.rng.standard_normal((2048, num_classes)) *
                                       np.sqrt(1.0 / 2048)).astype(np.float32))
    b = gb.constant("Logits/biases", np.zeros(num_classes, dtype=np.float32))
    logits = gb.bias_add(gb.matmul(x, w, name="Logits/MatMul"), b, name="logits")
    probs = gb.softmax(logits, name="probs")
    gb.top_k(probs, top_k, name="top_k")
    return gb.build_graph_def()


def inception_v3_flops_per_image(hw: int = 299) -> float:
    """Forward FLOPs (2·MAC) of Inception-v3 at hw×hw (≈5.7 GMAC at 299)."""
    return 5.72e9 * 2 * (hw / 299) ** 2
