"""FP8 (OCP e4m3fn) path: quantisation, fp8 MFMA conv/GEMM/pool kernels against fp32
references with the same quantisation points, and the Inception-v3 fp8 compiled plan
(calibrated scales, concat-by-stride-write in fp8) against the bf16 plan."""
import pytest
import torch
import torch.nn.functional as F

from flink_tensorflow_amd.graph.compiler import CompiledFunction
from flink_tensorflow_amd.graph.graph import Graph
from flink_tensorflow_amd.graph.session import Session
from flink_tensorflow_amd.models.zoo.inception_v3 import inception_v3_graph_def
from flink_tensorflow_amd.ops import fp8 as Q


def test_quantize_roundtrip_and_saturation():
    x = torch.tensor([0.0, 0.1, 1.0, 447.0, 1e4, -1e4, -3.3])
    b = Q.to_fp8_bytes(x)
    y = Q.from_fp8_bytes(b)
    assert y[4] == 448 and y[5] == -448  # saturating, never NaN
    assert (y[:4] - x[:4]).abs().max() <= 0.0625 * x[:4].abs().max()
    w = torch.randn(16, 3, 3, 32)
    wq, ws = Q.quantize_weight(w)
    assert wq.dtype == torch.uint8 and wq.shape == (16, 288) and ws.shape == (16,)
    back = Q.from_fp8_bytes(wq) * ws[:, None]
    assert ((back - w.reshape(16, -1)).abs() / w.reshape(16, -1).abs().amax(1, keepdim=True)).max() < 0.07


def test_conv_fp8_host_reference_tracks_fp32():
    torch.manual_seed(0)
    x = torch.randn(2, 9, 9, 32).relu()
    w = torch.randn(48, 3, 3, 32) * 0.1
    b = torch.randn(48) * 0.1
    sx = Q.scale_for(x.abs().max())
    wq, ws = Q.quantize_weight(w)
    y = Q.conv2d_nhwc_fp8(Q.quantize(x, sx), sx, wq, (3, 3), ws, b, (2, 2), (1, 1, 1, 1), act="relu")
    ref = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), b, 2, 1).relu().permute(0, 2, 3, 1)
    assert (y - ref).abs().max() < 0.08 * ref.abs().max()


def test_lite_fp8_tile_choice():
    """conv_lite_fp8's channel tile (kernels/fp8.hip ``lite_fp8_bn``; host logic, no GPU):
    the one of 192 / 160 / 128 / 96 / 64 that stages the fewest rows per 128-pixel tile,
    (Cout / BN tiles) x (128 + BN), ties to the wider tile."""
    from flink_tensorflow_amd import _ext

    hip = _ext.hip(required=False)
    if hip is None:
        pytest.skip("HIP kernel library not built")
    t = hip.lite_fp8_tile
    assert [t(c) for c in (80, 128, 160, 192, 288, 320, 448, 768)] == [96, 128, 160, 192, 160, 160, 160, 192]
    assert [t(c) for c in (64, 96, 384)] == [64, 96, 192]


def _inception_plans(device, hw=75, batch=2, **kw):
    g = Graph.from_graph_def(inception_v3_graph_def(image_hw=(hw, hw), out_hw=(hw, hw)))
    feeds = {"images:0": ((batch, hw, hw, 3), "UINT8")}
    fetch = ["logits:0", "top_k:1"]
    p16 = CompiledFunction(g, feeds, fetch, device, strict=True, **kw)
    p8 = CompiledFunction(g, feeds, fetch, device, strict=True, precision="fp8", **kw)
    return g, p16, p8


def test_inception_v3_fp8_plan_host():
    g, p16, p8 = _inception_plans("cpu")
    s8 = p8.summary()
    assert s8["glue_ops"] == [] and s8["fp8_layers"] == 93
    # every AvgPool(3x3/1) -> 1x1 conv branch runs as 1x1 conv -> pool (+ bias/ReLU/quantise)
    assert s8["commuted_pools"] == 9 and p16.summary()["commuted_pools"] == 9
    # each module's sibling 1x1 convs (and its commuted pool branch) run as one multi-output GEMM
    assert s8["sibling_groups"] == 10 and p16.summary()["sibling_groups"] == 0
    assert "concat" not in s8["kinds"] and "dequant" not in s8["kinds"]  # stride-written fp8 concats
    img = torch.randint(0, 256, (2, 75, 75, 3), dtype=torch.uint8)
    l16, _ = p16({"images:0": img})
    l8, _ = p8({"images:0": img})
    assert F.cosine_similarity(l16.flatten(), l8.flatten(), dim=0) > 0.99
    # the bf16 plan itself matches the op-by-op interpreter
    ref = Session(g).run(["logits:0"], {"images:0": img})[0]
    assert F.cosine_similarity(l16.flatten(), ref.flatten().float(), dim=0) > 0.999


# ------------------------------------------------------------------------------ GPU
DEV = torch.device("cuda", 0)


def _conv_case(cin, cout, k, stride, pads, in_bf16, out_fp8, cfg, offset=0, extra=0, N=2, H=11, W=13):
    kh, kw = (k, k) if isinstance(k, int) else k
    torch.manual_seed(cin + cout + kh * 7 + kw + cfg)
    x = torch.randn(N, H, W, cin).relu()
    w = torch.randn(cout, kh, kw, cin) / (kh * kw * cin) ** 0.5
    b = torch.randn(cout) * 0.1
    sx = Q.scale_for(x.abs().max())
    wq, ws = Q.quantize_weight(w)
    xin = x.to(torch.bfloat16) if in_bf16 else Q.quantize(x, sx)
    if in_bf16:  # the host reference quantises the same bf16 values
        x_host = xin.float()
    else:
        x_host = xin
    so = 0.02 if out_fp8 else None
    ref = Q.conv2d_nhwc_fp8(x_host, sx, wq, (kh, kw), ws, b, (stride, stride), pads, act="relu", out_scale=so)
    Ho, Wo = ref.shape[1:3]
    odt = torch.uint8 if out_fp8 else torch.bfloat16
    out = torch.zeros((N, Ho, Wo, cout + extra), dtype=odt, device=DEV)
    got = Q.conv2d_nhwc_fp8(xin.to(DEV), sx, wq.to(DEV), (kh, kw), ws.to(DEV), b.to(DEV), (stride, stride), pads,
                            act="relu", out_scale=so, out=out, out_channel_offset=offset, cfg=cfg)
    torch.cuda.synchronize()
    g = got[..., offset:offset + cout].cpu()
    if out_fp8:
        gd, rd = Q.from_fp8_bytes(g.contiguous()) * so, Q.from_fp8_bytes(ref) * so
        # accumulation order may flip a rounding tie: allow one e4m3 step (2^-3 relative)
        assert ((gd - rd).abs() <= 0.13 * rd.abs() + 1e-3).all()
        assert (gd == rd).float().mean() > 0.97
        if extra:
            assert (got[..., :offset] == 0).all() and (got[..., offset + cout:] == 0).all()
    else:
        torch.testing.assert_close(g.float(), ref.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 11])
def test_conv_fp8_configs_gpu(cfg):
    _conv_case(32, 64, 3, 1, (1, 1, 1, 1), False, True, cfg)
    _conv_case(64, 192, 3, 2, (0, 0, 0, 0), False, False, cfg)
    _conv_case(48, 96, (1, 7), 1, (0, 0, 3, 3), False, True, cfg, offset=32, extra=64)


@pytest.mark.gpu
@pytest.mark.parametrize("c", [11])
def test_conv_fp8_lite_shapes_gpu(c):
    """conv_lite_fp8 (cfg 11, the LDS-DMA tile the compiler uses; the other tiles were
    measured slower and removed): Cin not a multiple of the 128-byte K-tile (288,
    192, 80), K tails, Cout tails, 1x1 / 7x1 / strided, fp8 and bf16 output at a concat offset."""
    _conv_case(288, 384, 3, 2, (0, 0, 0, 0), False, True, c, N=2, H=17, W=17)
    _conv_case(192, 80, (7, 1), 1, (3, 3, 0, 0), False, False, c, N=3, H=9, W=9)
    _conv_case(80, 192, 3, 1, (1, 1, 1, 1), False, True, c, offset=64, extra=128)
    _conv_case(768, 128, 1, 1, (0, 0, 0, 0), False, True, c, N=4, H=9, W=9)
    _conv_case(16, 32, 3, 1, (1, 1, 1, 1), False, False, c)
    # channel tile 64 (Cout % 128 in (0, 64]) and the single-stage K <= 128 variants
    _conv_case(64, 80, 1, 1, (0, 0, 0, 0), False, True, c, N=3, H=13, W=13)      # K 64: one stage, BN 128
    _conv_case(64, 192, 1, 1, (0, 0, 0, 0), False, True, c, offset=64, extra=128)  # one stage, BN 64
    _conv_case(32, 320, 3, 1, (1, 1, 1, 1), False, False, c)                     # BN 64, 5 tiles
    _conv_case(128, 448, 1, 1, (0, 0, 0, 0), False, True, c, N=2, H=9, W=9)      # K 128 exactly, BN 64
    _conv_case(96, 96, 3, 1, (1, 1, 1, 1), False, True, c, offset=32, extra=64)   # BN 96
    _conv_case(48, 160, (1, 7), 1, (0, 0, 3, 3), False, False, c, N=2, H=9, W=9)  # BN 96, 2 tiles
    # the 192-wide tile: Cout 192 / 384, a Cout tail (160) and a concat offset
    _conv_case(160, 192, (7, 1), 1, (3, 3, 0, 0), False, True, c, N=2, H=17, W=17)
    _conv_case(288, 384, 3, 1, (1, 1, 1, 1), False, False, c, N=1, H=9, W=9)
    _conv_case(192, 160, (1, 7), 1, (0, 0, 3, 3), False, True, c, offset=32, extra=64, N=2, H=9, W=9)
    # ... and the 160-wide tile (the fewest staged rows: 320 = 2 x 160, 448 = 3 x 160)
    _conv_case(1280, 320, 1, 1, (0, 0, 0, 0), False, True, c, N=2, H=8, W=8)
    _conv_case(448, 448, (1, 3), 1, (0, 0, 1, 1), False, False, c, N=2, H=8, W=8)
    # long K walks (the per-lane tap / channel walk over 65-74 K-tiles)
    _conv_case(1040, 64, 3, 1, (1, 1, 1, 1), False, True, c, N=1, H=7, W=7)       # 74 K-tiles
    _conv_case(8320, 96, 1, 1, (0, 0, 0, 0), False, False, c, N=1, H=5, W=5)      # 65 K-tiles


@pytest.mark.gpu
def test_conv_fp8_pointwise_and_bf16_input_gpu():
    _conv_case(160, 128, 1, 1, (0, 0, 0, 0), False, True, -1, N=3, H=17, W=17)
    _conv_case(32, 32, 3, 1, (0, 0, 0, 0), True, True, -1)  # stem output (bf16) quantised on load
    _conv_case(32, 80, 3, 2, (0, 1, 0, 1), True, False, -1)


@pytest.mark.gpu
def test_gemm_fp8_gpu():
    torch.manual_seed(1)
    x = torch.randn(300, 256)
    w = torch.randn(96, 256) / 16
    sx = Q.scale_for(x.abs().max())
    wq, ws = Q.quantize_weight(w)
    ref = Q.gemm_fp8(Q.quantize(x, sx), sx, wq, ws, act=None)
    got = Q.gemm_fp8(Q.quantize(x, sx).to(DEV), sx, wq.to(DEV), ws.to(DEV), act=None)
    torch.testing.assert_close(got.float().cpu(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_quantize_dequantize_bitexact_gpu():
    x = (torch.randn(4096) * 30).to(torch.bfloat16)
    ref = Q.quantize(x.float(), 0.5)
    got = Q.quantize(x.to(DEV), 0.5).cpu()
    assert torch.equal(got, ref)
    back = Q.dequantize(got.to(DEV), 0.5).cpu()
    assert torch.equal(back, (Q.from_fp8_bytes(ref) * 0.5).to(torch.bfloat16))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["max", "avg"])
def test_pool_fp8_gpu(mode):
    torch.manual_seed(2)
    x = Q.quantize(torch.randn(2, 9, 9, 48).relu(), 0.01)
    for ks, st, pad in (((3, 3), (1, 1), (1, 1, 1, 1)), ((3, 3), (2, 2), (0, 0, 0, 0))):
        ref = Q.pool2d_nhwc_fp8(x, ks, st, pad, mode, rq=0.7)
        got = Q.pool2d_nhwc_fp8(x.to(DEV), ks, st, pad, mode, rq=0.7).cpu()
        gd, rd = Q.from_fp8_bytes(got), Q.from_fp8_bytes(ref)
        assert ((gd - rd).abs() <= 0.13 * rd.abs() + 1e-6).all(), mode
    ref = Q.global_avgpool_fp8(x, 0.01)
    got = Q.global_avgpool_fp8(x.to(DEV), 0.01).float().cpu()
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-3)


@pytest.mark.gpu
def test_maxpool3_fp8_unrolled_gpu():
    """The unrolled 3x3 / row-stride-2 max pool (Inception's stem and grid-reduction pools):
    odd widths (an odd output count leaves the thread's second output unused), SAME and
    VALID padding, column stride 1 and 2, signed inputs (padding must not win the max),
    16..192 channels, a requantising rq and a channel offset into a wider buffer."""
    torch.manual_seed(3)
    for (N, H, W, C), pad, st in (((2, 15, 15, 64), (0, 0, 0, 0), (2, 2)),
                                  ((3, 9, 13, 192), (1, 1, 1, 1), (2, 2)),
                                  ((1, 8, 10, 16), (0, 1, 0, 1), (2, 2)),
                                  ((2, 11, 7, 48), (1, 1, 1, 1), (2, 1))):
        x = Q.quantize(torch.randn(N, H, W, C) * 3 - 1, 0.05)  # mostly negative
        ref = Q.pool2d_nhwc_fp8(x, (3, 3), st, pad, "max")
        got = Q.pool2d_nhwc_fp8(x.to(DEV), (3, 3), st, pad, "max").cpu()
        assert torch.equal(got, ref), (N, H, W, C, pad, st)  # rq 1: the max is one of the input bytes
        ref = Q.pool2d_nhwc_fp8(x, (3, 3), st, pad, "max", rq=0.8)
        got = Q.pool2d_nhwc_fp8(x.to(DEV), (3, 3), st, pad, "max", rq=0.8).cpu()
        gd, rd = Q.from_fp8_bytes(got), Q.from_fp8_bytes(ref)
        assert ((gd - rd).abs() <= 0.13 * rd.abs() + 1e-6).all() and (got == ref).float().mean() > 0.99
    x = Q.quantize(torch.randn(2, 13, 13, 32).relu(), 0.02)
    ref = Q.pool2d_nhwc_fp8(x, (3, 3), (2, 2), (0, 0, 0, 0), "max")
    out = torch.zeros((2, 6, 6, 96), dtype=torch.uint8, device=DEV)
    Q.pool2d_nhwc_fp8(x.to(DEV), (3, 3), (2, 2), (0, 0, 0, 0), "max", out=out, out_channel_offset=32)
    torch.cuda.synchronize()
    assert torch.equal(out[..., 32:64].cpu(), ref)
    assert (out[..., :32] == 0).all() and (out[..., 64:] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("out_fp8", [True, False])
def test_avgpool_bias_act_gpu(out_fp8):
    """The pool half of a commuted AvgPool -> 1x1 conv branch: bf16 in, TF SAME average,
    bias + ReLU, fp8 (or bf16) into a concat slot; against the fp32 host reference."""
    torch.manual_seed(4)
    x = (torch.randn(3, 17, 17, 64) * 2).to(torch.bfloat16)
    b = torch.randn(64) * 0.5
    so = 0.02 if out_fp8 else None
    for ks, st, pad in (((3, 3), (1, 1), (1, 1, 1, 1)), ((3, 3), (2, 2), (0, 0, 0, 0)),
                        ((3, 3), (1, 1), (0, 0, 0, 0)), ((3, 3), (1, 1), (1, 0, 0, 1))):
        ref = Q.avgpool_bias_act(x.float(), ks, st, pad, b, "relu", out_scale=so)
        Ho, Wo = ref.shape[1:3]
        out = torch.zeros((3, Ho, Wo, 96), dtype=torch.uint8 if out_fp8 else torch.bfloat16, device=DEV)
        Q.avgpool_bias_act(x.to(DEV), ks, st, pad, b.to(DEV), "relu", out_scale=so, out=out, out_channel_offset=32)
        got = out.cpu()
        assert (got[..., :32] == 0).all()
        if out_fp8:
            gd, rd = Q.from_fp8_bytes(got[..., 32:].contiguous()) * so, Q.from_fp8_bytes(ref) * so
            assert ((gd - rd).abs() <= 0.13 * rd.abs() + 1e-3).all()
        else:
            torch.testing.assert_close(got[..., 32:].float(), ref.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("C", [96, 192])
def test_conv_fp8_multi_output_gpu(C):
    """Sibling 1x1 convs as one GEMM with a multi-destination epilogue: fp8 segments of
    different scales (one at a concat offset), a bf16 segment, ReLU and no-act channels;
    against the host reference of the same kernel.  C 192 takes the two-stage tile."""
    torch.manual_seed(6)
    N, H, W = 2, 13, 11
    x = torch.randn(N, H, W, C).relu()
    sx = Q.scale_for(x.abs().max())
    xq = Q.quantize(x, sx)
    couts = (64, 48, 32, 16)
    w = torch.randn(sum(couts), C) / C ** 0.5
    wq, ws = Q.quantize_weight(w)
    b = torch.randn(sum(couts)) * 0.1
    lo = torch.tensor([0.0] * (64 + 48) + [float("-inf")] * 48)

    def outs(dev):
        return [torch.zeros((N, H, W, 128), dtype=torch.uint8, device=dev),   # concat slot at 32
                torch.zeros((N, H, W, 48), dtype=torch.uint8, device=dev),
                torch.zeros((N, H, W, 32), dtype=torch.bfloat16 if dev != "cpu" else torch.float32, device=dev),
                torch.zeros((N, H, W, 16), dtype=torch.uint8, device=dev)]

    def segs(o):
        return [(o[0], 0, 64, 32, 0.02), (o[1], 64, 112, 0, 0.05), (o[2], 112, 144, 0, None), (o[3], 144, 160, 0, 0.01)]

    ref = outs("cpu")
    Q.conv2d_nhwc_fp8_multi(xq, sx, wq, (1, 1), ws, b, lo, segs(ref))
    got = outs(DEV)
    Q.conv2d_nhwc_fp8_multi(xq.to(DEV), sx, wq.to(DEV), (1, 1), ws.to(DEV), b.to(DEV), lo.to(DEV), segs(got))
    torch.cuda.synchronize()
    for i, (r, g) in enumerate(zip(ref, got)):
        g = g.cpu()
        if r.dtype == torch.uint8:
            rd, gd = Q.from_fp8_bytes(r), Q.from_fp8_bytes(g)
            assert ((gd - rd).abs() <= 0.13 * rd.abs() + 0.02).all(), i  # raw e4m3 units: subnormal ties
        else:
            torch.testing.assert_close(g.float(), r.float(), rtol=2e-2, atol=2e-2)
    assert (got[0][..., :32] == 0).all() and (got[0][..., 96:] == 0).all()
    assert (Q.from_fp8_bytes(got[3].cpu()) < 0).any()  # the no-act channels keep their negatives


@pytest.mark.gpu
def test_inception_v3_fp8_plan_gpu():
    g = Graph.from_graph_def(inception_v3_graph_def(image_hw=(75, 75), out_hw=(75, 75)))
    feeds = {"images:0": ((4, 75, 75, 3), "UINT8")}
    img = torch.randint(0, 256, (4, 75, 75, 3), dtype=torch.uint8, generator=torch.Generator().manual_seed(5))
    calib = {"images:0": img}
    host = CompiledFunction(g, feeds, ["logits:0"], "cpu", strict=True, precision="fp8", calibration=calib)
    dev = CompiledFunction(g, feeds, ["logits:0"], DEV, strict=True, precision="fp8", calibration=calib)
    assert dev.summary()["hip_graph"] and dev.summary()["fp8_layers"] == 93
    # Conv2d_2b + MaxPool_3a stay apart: the pooled tiling would waste > 15 % of the conv work
    assert dev.summary()["fused_pools"] == 0
    assert dev.summary()["fused_preprocess"] == 1  # Conv2d_1a reads the raw uint8 batch
    lh = host({"images:0": img})[0]
    ld = dev({"images:0": img.to(DEV)})[0].cpu()
    assert F.cosine_similarity(lh.flatten(), ld.flatten(), dim=0) > 0.99


@pytest.mark.gpu
def test_stem_from_raw_uint8_equals_preprocess_then_conv_gpu():
    """The s2d RGB stem built straight from the raw uint8 batch (``dconv_u8s2d``, the
    resize-free preprocess folded in) equals the preprocess kernel's s2d output fed to the
    same direct conv, bit for bit (odd image size: the last block row / column is zero).
    (Folding a bilinear resize in as well — ResNet-50's stem — measured slower: 249 µs vs
    49 + 164 µs, profiles/r05_g.)"""
    from flink_tensorflow_amd.ops import kernels as K

    torch.manual_seed(2)
    N, Hi, Wi, Cout = 3, 37, 35, 32
    x = torch.randint(0, 256, (N, Hi, Wi, 3), dtype=torch.uint8)
    w = torch.randn(3, 3, 3, Cout) / 4
    b = torch.randn(Cout) * 0.1
    w2, bp = K.s2d_stem_weights(w, Hi, Wi, (0, 0, 0, 0))
    w_arr = K.dconv_bf16_weight_bytes(w2, 32).to(DEV)
    mean, std = (128.0, 120.0, 110.0), (64.0, 60.0, 70.0)
    xs = K.preprocess_images(x.to(DEV), (Hi, Wi), mean, std, s2d=True)
    ref = K.conv2d_direct(xs, w_arr, (2, 2), Cout, b.to(DEV), (1, 1), bp, "relu", bn=32, out_scale=0.05)
    got = K.conv2d_direct_u8s2d(x.to(DEV), w_arr, (2, 2), Cout, b.to(DEV), bp, "relu", mean, std, bn=32,
                                out_scale=0.05)
    assert torch.equal(got, ref)
