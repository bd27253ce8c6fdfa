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
    assert len(fused.steps) == len(plain.steps) - n
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


def _chain_case(dev, M_hw=(2, 6, 10)):
    """Three stage-1 tails unfused (``bottleneck_tail``: dual, then two identity-residual
    ones reading the previous y3) against the recomputing chains (``bottleneck_chain``
    with 1, 2 and 3 links): the same y1 of every tail and the same (decimated) last y3."""
    g = torch.Generator().manual_seed(9)
    N, H, W = M_hw

    def bf(*shape, s=1.0):
        return (torch.randn(*shape, generator=g) * s).bfloat16().float()

    x0, c1, c2, c3 = (bf(N, H, W, 64) for _ in range(4))
    wa, wb, wc = bf(256, 128, s=1 / 11), bf(256, 64, s=1 / 8), bf(256, 64, s=1 / 8)
    ba, bb, bc = (torch.randn(256, generator=g) * 0.1 for _ in range(3))
    w1a, w1b, w1c = bf(64, 256, s=1 / 16), bf(64, 256, s=1 / 16), bf(128, 256, s=1 / 16)
    b1a, b1b, b1c = torch.randn(64, generator=g), torch.randn(64, generator=g), torch.randn(128, generator=g)
    cast = (lambda t: t.to(dev, torch.bfloat16)) if dev.type == "cuda" else (lambda t: t)
    fp = (lambda t: t.to(dev)) if dev.type == "cuda" else (lambda t: t)
    # unfused: three tails, y3 round-tripping
    y3a, y1a = K.bottleneck_tail(cast(c1), None, cast(wa), fp(ba), cast(w1a), fp(b1a), xs=cast(x0))
    y3b, y1b = K.bottleneck_tail(cast(c2), y3a, cast(wb), fp(bb), cast(w1b), fp(b1b))
    y3c, y1c = K.bottleneck_tail(cast(c3), y3b, cast(wc), fp(bc), cast(w1c), fp(b1c), y3_decimated=True)
    la = (cast(c1), cast(x0), cast(wa), fp(ba))
    lb = (cast(c2), None, cast(wb), fp(bb))
    lc = (cast(c3), None, cast(wc), fp(bc))
    n1, z1 = K.bottleneck_chain([la], cast(w1a), fp(b1a), store_y3=False)
    n2, z2 = K.bottleneck_chain([la, lb], cast(w1b), fp(b1b), store_y3=False)
    z3c, z3 = K.bottleneck_chain([la, lb, lc], cast(w1c), fp(b1c), y3_decimated=True)
    assert n1 is None and n2 is None and tuple(z3c.shape) == (N, H // 2, W // 2, 256)
    # the chain rounds every link exactly as the tails do: bit-identical
    for a, b in ((z1, y1a), (z2, y1b), (z3, y1c), (z3c, y3c)):
        assert torch.equal(a.float().cpu(), b.float().cpu())


def test_chain_reference_equals_unfused_tails():
    _chain_case(torch.device("cpu"))
    with pytest.raises(ValueError):  # the first link must be the dual one
        K.bottleneck_chain([(torch.zeros(2, 64), None, torch.zeros(256, 64), torch.zeros(256))], torch.zeros(64, 256),
                           torch.zeros(64))


@pytest.mark.gpu
def test_chain_kernel_equals_unfused_tails_gpu():
    _chain_case(torch.device("cuda", 0))
    _chain_case(torch.device("cuda", 0), (3, 8, 14))  # a partial last tile


def _compile_chain(g, dev, on, links=2):
    from flink_tensorflow_amd.config import override

    with override(recompute_tails=on, chain_max_links=links):
        return CompiledFunction(g, {"images:0": ((2, 64, 64, 3), "UINT8")}, ["logits:0"], dev, strict=True)


def _check_chain(r50, dev, links=2):
    on, off = _compile_chain(r50, dev, True, links), _compile_chain(r50, dev, False)
    # links 2 (default): tail 1 -> tail 2 chained, tail 3 reads y3; links 3: all three
    assert on.summary()["chained_tails"] == links - 1 and off.summary()["chained_tails"] == 0
    assert on.summary()["fused_tails"] == off.summary()["fused_tails"] == 3
    assert on.activation_bytes <= off.activation_bytes * 1.25
    imgs = torch.randint(0, 256, (2, 64, 64, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(2))
    a = on({"images:0": imgs.to(dev)})[0].float().cpu()
    b = off({"images:0": imgs.to(dev)})[0].float().cpu()
    assert torch.equal(a, b)  # the recomputed residual stream is bit-identical


@pytest.mark.parametrize("links", [2, 3])
def test_compiled_resnet50_recomputes_the_stage1_residual_stream_cpu(r50, links):
    _check_chain(r50, torch.device("cpu"), links)


@pytest.mark.gpu
@pytest.mark.parametrize("links", [2, 3])
def test_compiled_resnet50_recomputes_the_stage1_residual_stream_gpu(r50, links):
    _check_chain(r50, torch.device("cuda", 0), links)
