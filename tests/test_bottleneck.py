"""Fused ResNet stage-1 block boundary (``ops.kernels.bottleneck_tail``): the host
reference, and the compiler's fusion of a 1x1 expand conv with the next block's 1x1
reduce conv (three boundaries in ResNet-50: the two inside stage 1 — the first one with the
projection shortcut folded in — and stage 1 -> stage 2), and the GEMM lowering of the
deep-K 1x1 convs (GPU)."""
import os

import pytest
import torch

from flink_tensorflow_amd.graph.compiler import CompiledFunction
from flink_tensorflow_amd.graph.graph import Graph
from flink_tensorflow_amd.models.zoo.resnet import resnet50_graph_def
from flink_tensorflow_amd.ops import kernels as K


def test_host_reference_matches_two_convs():
    g = torch.Generator().manual_seed(0)
    x2, res = torch.randn(2, 5, 7, 64, generator=g), torch.randn(2, 5, 7, 256, generator=g)
    w3, w1 = torch.randn(256, 64, generator=g), torch.randn(128, 256, generator=g)
    b3, b1 = torch.randn(256, generator=g), torch.randn(128, generator=g)
    y3, y1 = K.bottleneck_tail(x2, res, w3, b3, w1, b1)
    e3 = K.conv2d_nhwc(x2, w3.reshape(256, 1, 1, 64), b3, res, act="relu")
    e1 = K.conv2d_nhwc(e3, w1.reshape(128, 1, 1, 256), b1, act="relu")
    torch.testing.assert_close(y3, e3)
    torch.testing.assert_close(y1, e1, rtol=1e-4, atol=1e-3)
    with pytest.raises(ValueError):
        K.bottleneck_tail(x2, res, w3, b3, w1[:96], b1[:96])
    # dual form: expand + stride-1 projection shortcut over [x2 | xs], no residual
    xs, wsc = torch.randn(2, 5, 7, 64, generator=g), torch.randn(256, 64, generator=g)
    w1 = w1[:64]
    y3, y1 = K.bottleneck_tail(x2, None, torch.cat([w3, wsc], 1), b3, w1, b1[:64], xs=xs)
    e3 = torch.relu(K.conv2d_nhwc(x2, w3.reshape(256, 1, 1, 64), b3) + K.conv2d_nhwc(xs, wsc.reshape(256, 1, 1, 64)))
    e1 = K.conv2d_nhwc(e3, w1.reshape(64, 1, 1, 256), b1[:64], act="relu")
    torch.testing.assert_close(y3, e3, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(y1, e1, rtol=1e-4, atol=1e-3)
    # the stage-2 form (128 -> 512 -> 128, weights streamed through LDS) was removed
    with pytest.raises(ValueError):
        K.bottleneck_tail(torch.randn(3, 4, 128), torch.randn(3, 4, 512), torch.randn(512, 128), torch.randn(512),
                          torch.randn(128, 512), torch.randn(128))


def _compile(g, dev, fuse):
    from flink_tensorflow_amd.config import override

    with override(fuse_block_tails=fuse):
        return CompiledFunction(g, {"images:0": ((2, 64, 64, 3), "UINT8")}, ["logits:0"], dev, strict=True)


@pytest.fixture(scope="module")
def r50():
    return Graph.from_graph_def(resnet50_graph_def(depth=50, image_hw=(64, 64), num_classes=16))


def _check(r50, dev):
    fused, plain = _compile(r50, dev, True), _compile(r50, dev, False)
    # stage 1: block 1 (dual: projection shortcut) -> 2 -> 3 -> stage 2 block 1
    n = 3
    assert fused.summary()["fused_tails"] == n and plain.summary()["fused_tails"] == 0
    assert fused.summary()["fused_shortcuts"] == plain.summary()["fused_shortcuts"] == 4
    # stage 1 -> stage 2: the tail's 256-channel output is stored decimated (only the
    # stride-2 projection reads it besides the fused reduce conv)
    assert fused.summary()["decimated_tails"] == 1 and plain.summary()["decimated_tails"] == 0
    # on the GPU the three stage-1 3x3 convs also join their tails (bottleneck3)
    c3 = fused.summary()["fused_conv3_tails"]
    assert c3 == (3 if dev.type == "cuda" else 0) and plain.summary()["fused_conv3_tails"] == 0
    assert len(fused.steps) == len(plain.steps) - n - c3
    # deep-K 1x1 reduce convs (stages 3/4) run on the ping-pong GEMM on the GPU; the FC head
    # too; no library GEMM anywhere
    for plan in (fused, plain):
        kinds = plan.summary()["kinds"]
        assert "gemm_lib" not in kinds
        # 9 deep-K reduce convs + the stage-3 entry reduce (K 512 -> 256) + FC on the GPU
        assert kinds.get("gemm", 0) == (10 if dev.type == "cuda" else 1)
    imgs = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(1))
    a = fused({"images:0": imgs.to(dev)})[0].float().cpu()
    b = plain({"images:0": imgs.to(dev)})[0].float().cpu()
    torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2 * b.abs().max().item())


def test_compiled_resnet50_fuses_block_boundaries_cpu(r50):
    _check(r50, torch.device("cpu"))


@pytest.mark.gpu
def test_compiled_resnet50_fuses_block_boundaries_gpu(r50):
    _check(r50, torch.device("cuda", 0))


def _decimated_case(dev):
    g = torch.Generator().manual_seed(5)
    x2, res = torch.randn(2, 6, 10, 64, generator=g), torch.randn(2, 6, 10, 256, generator=g)
    w3, w1 = torch.randn(256, 64, generator=g) / 8, torch.randn(128, 256, generator=g) / 16
    b3, b1 = torch.randn(256, generator=g), torch.randn(128, generator=g)
    x2, res, w3, w1 = (t.bfloat16().float() for t in (x2, res, w3, w1))  # exact in bf16
    full3, full1 = K.bottleneck_tail(x2, res, w3, b3, w1, b1)
    cast = (lambda t: t.to(dev, torch.bfloat16)) if dev.type == "cuda" else (lambda t: t)
    fp = (lambda t: t.to(dev)) if dev.type == "cuda" else (lambda t: t)
    y3, y1 = K.bottleneck_tail(cast(x2), cast(res), cast(w3), fp(b3), cast(w1), fp(b1), y3_decimated=True)
    assert tuple(y3.shape) == (2, 3, 5, 256) and tuple(y1.shape) == (2, 6, 10, 128)
    tol = dict(rtol=3e-2, atol=3e-2 * full3.abs().max().item()) if dev.type == "cuda" else {}
    torch.testing.assert_close(y3.float().cpu(), full3[:, ::2, ::2], **tol)
    tol1 = dict(rtol=3e-2, atol=3e-2 * full1.abs().max().item()) if dev.type == "cuda" else {}
    torch.testing.assert_close(y1.float().cpu(), full1, **tol1)


def test_decimated_tail_reference():
    """y3_decimated stores only the even-(h, w) pixels of y3, compact; y1 is unchanged."""
    _decimated_case(torch.device("cpu"))
    with pytest.raises(ValueError):
        K.bottleneck_tail(torch.zeros(1, 5, 4, 64), torch.zeros(1, 5, 4, 256), torch.zeros(256, 64), torch.zeros(256),
                          torch.zeros(128, 256), torch.zeros(128), y3_decimated=True)  # odd H


@pytest.mark.gpu
def test_decimated_tail_gpu():
    _decimated_case(torch.device("cuda", 0))


def _b3_case(g, N, H, W, dual, cn):
    y1 = torch.randn(N, H, W, 64, generator=g).relu()
    w2 = torch.randn(64, 3, 3, 64, generator=g) / 24
    b2 = torch.randn(64, generator=g) * 0.1
    w3 = torch.randn(256, 128 if dual else 64, generator=g) / 8
    b3 = torch.randn(256, generator=g) * 0.1
    w1 = torch.randn(cn, 256, generator=g) / 16
    b1 = torch.randn(cn, generator=g) * 0.1
    second = torch.randn(N, H, W, 64 if dual else 256, generator=g)
    return y1, w2, b2, w3, b3, w1, b1, second


def test_bottleneck3_host_reference():
    """bottleneck3 = the 3x3 conv (+ bias, ReLU) then the block tail, on the host path."""
    g = torch.Generator().manual_seed(3)
    for dual, cn in ((True, 64), (False, 64), (False, 128)):
        y1, w2, b2, w3, b3, w1, b1, second = _b3_case(g, 2, 5, 7, dual, cn)
        y3, y1o = K.bottleneck3(y1, w2, b2, None if dual else second, w3, b3, w1, b1, xs=second if dual else None)
        x2 = K.conv2d_nhwc(y1, w2, b2, None, (1, 1), (1, 1, 1, 1), (1, 1), "relu")
        e3, e1 = K.bottleneck_tail(x2, None if dual else second, w3, b3, w1, b1, xs=second if dual else None)
        torch.testing.assert_close(y3, e3)
        torch.testing.assert_close(y1o, e1)
    with pytest.raises(ValueError):
        K.bottleneck3(y1, w2[:32], b2, second, w3, b3, w1, b1)


B3_CASES = [  # N, H, W, dual, cn, decimated
    (3, 56, 56, True, 64, False),    # stage 1's first block (projection shortcut)
    (3, 56, 56, False, 64, False),
    (3, 56, 56, False, 128, True),   # stage 1 -> stage 2: y3 stored decimated
    (2, 10, 40, False, 64, False),   # partial tiles: a 12-column last tile
    (2, 12, 34, False, 128, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", B3_CASES)
def test_bottleneck3_matches_unfused_gpu(case):
    """The fused kernel equals conv3x3c64 followed by bottleneck_tail up to bf16 rounding
    flips (its 3x3 sums two K halves in fp32; everything after x2 is the tail's arithmetic)."""
    N, H, W, dual, cn, dec = case
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(N * H + W + cn)
    y1, w2, b2, w3, b3, w1, b1, second = (t.to(dev) for t in _b3_case(g, N, H, W, dual, cn))
    bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    y1, w2, w3, w1, second = bf(y1), bf(w2), bf(w3), bf(w1), bf(second)
    x2 = K.conv3x3_c64(y1, w2, b2, "relu")
    e3, e1 = K.bottleneck_tail(x2, None if dual else second, w3, b3, w1, b1, xs=second if dual else None,
                               y3_decimated=dec)
    y3, y1o = K.bottleneck3(y1, w2, b2, None if dual else second, w3, b3, w1, b1, xs=second if dual else None,
                            y3_decimated=dec)
    torch.cuda.synchronize()
    for got, ref in ((y3, e3), (y1o, e1)):
        g32, r32 = got.float(), ref.float()
        torch.testing.assert_close(g32, r32, rtol=2e-2, atol=2e-2 * r32.abs().max().item())
        assert (g32 == r32).float().mean() > 0.9
    # and against the fp32 host reference
    r3, r1 = K.bottleneck3(y1.float().cpu(), w2.float().cpu(), b2.cpu(), None if dual else second.float().cpu(),
                           w3.float().cpu(), b3.cpu(), w1.float().cpu(), b1.cpu(),
                           xs=second.float().cpu() if dual else None, y3_decimated=dec)
    torch.testing.assert_close(y3.float().cpu(), r3, rtol=3e-2, atol=3e-2 * r3.abs().max().item())
    torch.testing.assert_close(y1o.float().cpu(), r1, rtol=3e-2, atol=3e-2 * r1.abs().max().item())


@pytest.mark.gpu
def test_bottleneck3_odd_shape_gpu():
    """Shapes conv3x3c64 does not take (H < 8, W < 32, odd): against the fp32 reference."""
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(11)
    y1, w2, b2, w3, b3, w1, b1, res = _b3_case(g, 2, 7, 30, False, 64)
    bf = lambda t: t.to(dev, torch.bfloat16).contiguous()  # noqa: E731
    y3, y1o = K.bottleneck3(bf(y1), bf(w2), b2.to(dev), bf(res), bf(w3), b3.to(dev), bf(w1), b1.to(dev))
    r3, r1 = K.bottleneck3(*(bf(t).float().cpu() for t in (y1, w2)), b2, bf(res).float().cpu(),
                           bf(w3).float().cpu(), b3, bf(w1).float().cpu(), b1)
    torch.testing.assert_close(y3.float().cpu(), r3, rtol=3e-2, atol=3e-2 * r3.abs().max().item())
    torch.testing.assert_close(y1o.float().cpu(), r1, rtol=3e-2, atol=3e-2 * r1.abs().max().item())


@pytest.mark.gpu
def test_compiled_resnet50_fuses_conv3_tails_gpu():
    """At 128x128 input (stage 1 at 32x32, where conv3x3c64 applies) the three stage-1
    3x3 convs join their block tails; logits match the unfused plan."""
    from flink_tensorflow_amd.config import override

    dev = torch.device("cuda", 0)
    r = Graph.from_graph_def(resnet50_graph_def(depth=50, image_hw=(128, 128), num_classes=16))
    plans = {}
    for on in (True, False):
        with override(fuse_conv3_tails=on):
            plans[on] = CompiledFunction(r, {"images:0": ((4, 128, 128, 3), "UINT8")}, ["logits:0"], dev, strict=True)
    assert plans[True].summary()["fused_conv3_tails"] == 3 and plans[False].summary()["fused_conv3_tails"] == 0
    assert len(plans[True].steps) == len(plans[False].steps) - 3
    assert sum(st.meta.get("impl") == "bottleneck3" for st in plans[True].steps) == 3
    imgs = torch.randint(0, 256, (4, 128, 128, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(2))
    a = plans[True]({"images:0": imgs.to(dev)})[0].float().cpu()
    b = plans[False]({"images:0": imgs.to(dev)})[0].float().cpu()
    torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2 * b.abs().max().item())
