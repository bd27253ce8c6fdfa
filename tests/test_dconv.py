"""Direct (LDS-resident) convolution kernel for narrow layers vs the fp32 references:
bf16 and fp8 inputs, stride 1/2, asymmetric padding, bf16/e4m3 outputs, concat slices."""
import pytest
import torch

from flink_tensorflow_amd.ops import fp8 as Q
from flink_tensorflow_amd.ops import kernels as K

DEV = torch.device("cuda", 0)


def test_dconv_eligibility_host():
    assert K.dconv_eligible(8, 3, 3, (2, 2), (1, 1), 2)
    assert K.dconv_eligible(32, 3, 3, (1, 1), (1, 1), 1)
    assert not K.dconv_eligible(48, 5, 5, (1, 1), (1, 1), 1)  # 48 B is not a 32-B lane segment multiple
    assert not K.dconv_eligible(64, 1, 1, (1, 1), (1, 1), 2)  # pointwise stays on the GEMM path
    w = torch.randn(40, 3, 3, 8)
    arr = K.dconv_bf16_weight_bytes(w, 32)
    assert arr.shape == (64, 9 * 8 * 2 + (64 - 144 % 64) % 64 + 16)


BF16_CASES = [  # N, H, W, Cin, Cout, (kh, kw), stride, pad, bn, out_fp8
    (2, 31, 31, 8, 32, (3, 3), 2, (0, 0, 0, 0), 32, False),
    (2, 31, 31, 8, 32, (3, 3), 2, (0, 0, 0, 0), 32, True),
    (2, 28, 28, 16, 64, (4, 4), 1, (1, 2, 1, 2), 64, False),
    (2, 19, 21, 64, 64, (3, 3), 1, (1, 1, 1, 1), 32, False),
    (1, 9, 40, 32, 48, (1, 7), 1, (0, 0, 3, 3), 64, False),
]


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("case", BF16_CASES)
def test_dconv_bf16_gpu(case, waves):
    N, H, W, Cin, Cout, (kh, kw), s, pad, bn, out_fp8 = case
    torch.manual_seed(hash(case) % 1000)
    x = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    w = (torch.randn(Cout, kh, kw, Cin) / (kh * kw * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout) * 0.1
    so = 0.01 if out_fp8 else None
    ref = K.conv2d_nhwc(x, w, b, None, (s, s), pad, (1, 1), "relu", out_scale=so)
    arr = K.dconv_bf16_weight_bytes(w.float(), bn).to(DEV)
    got = K.conv2d_direct(x.to(DEV), arr, (kh, kw), Cout, b.to(DEV), (s, s), pad, "relu", bn=bn, out_scale=so,
                          waves=waves).cpu()
    if out_fp8:
        gd, rd = Q.from_fp8_bytes(got), Q.from_fp8_bytes(ref)
        assert ((gd - rd).abs() <= 0.13 * rd.abs() + 1e-3).all()
    else:
        torch.testing.assert_close(got.float(), ref.float(), rtol=2e-2, atol=2e-2 * ref.abs().max().item())


FP8_CASES = [  # N, H, W, Cin, Cout, k, stride, pad, bn, offset, extra
    (2, 23, 23, 32, 32, 3, 1, (0, 0, 0, 0), 32, 0, 0),
    (2, 20, 17, 32, 64, 3, 1, (1, 1, 1, 1), 64, 0, 0),
    (2, 35, 35, 64, 96, 3, 1, (1, 1, 1, 1), 32, 32, 64),
    (2, 35, 35, 96, 96, 3, 1, (1, 1, 1, 1), 64, 0, 0),
    (2, 17, 17, 128, 128, (1, 7), 1, (0, 0, 3, 3), 64, 0, 0),
]


@pytest.mark.gpu
@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("case", FP8_CASES)
def test_dconv_fp8_gpu(case, waves):
    N, H, W, Cin, Cout, k, s, pad, bn, off, extra = case
    kh, kw = (k, k) if isinstance(k, int) else k
    torch.manual_seed(Cin * 7 + Cout + kh)
    x = torch.randn(N, H, W, Cin).relu()
    sx = Q.scale_for(x.max())
    xq = Q.quantize(x, sx)
    wq, ws = Q.quantize_weight(torch.randn(Cout, kh, kw, Cin) / (kh * kw * Cin) ** 0.5)
    b = torch.randn(Cout) * 0.1
    so = 0.02
    ref = Q.conv2d_nhwc_fp8(xq, sx, wq, (kh, kw), ws, b, (s, s), pad, act="relu", out_scale=so)
    Ho, Wo = ref.shape[1:3]
    out = torch.zeros((N, Ho, Wo, Cout + extra), dtype=torch.uint8, device=DEV)
    arr = K.dconv_weights(wq, Cout, 1, bn).to(DEV)
    K.conv2d_direct(xq.to(DEV), arr, (kh, kw), Cout, b.to(DEV), (s, s), pad, "relu", out=out, out_channel_offset=off,
                    bn=bn, chan_scale=(ws * sx).to(DEV), out_scale=so, waves=waves)
    got = out[..., off:off + Cout].cpu()
    gd, rd = Q.from_fp8_bytes(got.contiguous()), Q.from_fp8_bytes(ref)
    # raw e4m3 units: one step (2^-3 relative) of slack for accumulation-order rounding flips;
    # near zero the subnormal step is 2^-9, so allow a few of those absolutely
    bad = (gd - rd).abs() > 0.13 * rd.abs() + 0.02
    assert not bad.any(), (gd[bad][:8], rd[bad][:8])
    assert (gd == rd).float().mean() > 0.97
    if extra:
        assert (out[..., :off] == 0).all() and (out[..., off + Cout:] == 0).all()


POOL_CASES = [  # N, H, W, Cin, Cout, (kh, kw), stride, pad, pool padding (TF "SAME"/"VALID"), bn
    (2, 56, 56, 16, 64, (4, 4), 1, (2, 1, 2, 1), "SAME", 64),  # ResNet s2d stem at 1/2 scale
    (1, 45, 39, 8, 32, (3, 3), 1, (1, 1, 1, 1), "SAME", 32),  # odd sizes: pads 1/1
    (2, 33, 30, 16, 64, (3, 3), 1, (1, 1, 1, 1), "VALID", 64),
    (1, 30, 40, 16, 64, (4, 4), 1, (2, 1, 2, 1), "SAME", 64),  # partial last tile row and column
    (12, 112, 112, 16, 64, (4, 4), 1, (2, 1, 2, 1), "SAME", 64),  # the 224x224 ResNet s2d stem
]


@pytest.mark.gpu
@pytest.mark.parametrize("pool_rows", [7, 14])
@pytest.mark.parametrize("case", POOL_CASES)
def test_dconv_maxpool_gpu(case, pool_rows):
    """Stem conv + ReLU + fused 3x3/s2 max pool == conv then pool (the same bf16 values
    are compared inside the max, so the results are exact up to conv rounding); both pooled
    tile heights (7 rows / 4 waves, 14 rows / 8 waves)."""
    N, H, W, Cin, Cout, (kh, kw), s, pad, ppad, bn = case
    torch.manual_seed(H * W + Cin)
    x = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    w = (torch.randn(Cout, kh, kw, Cin) / (kh * kw * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout) * 0.1
    conv = K.conv2d_nhwc(x, w, b, None, (s, s), pad, (1, 1), "relu")
    Ho, Wo = conv.shape[1:3]
    if ppad == "SAME":
        ph = max((-(-Ho // 2) - 1) * 2 + 3 - Ho, 0)
        pw = max((-(-Wo // 2) - 1) * 2 + 3 - Wo, 0)
        mp = (ph // 2, ph - ph // 2, pw // 2, pw - pw // 2)
    else:
        mp = (0, 0, 0, 0)
    ref = K.pool2d_nhwc(conv, (3, 3), (2, 2), mp, "max")
    arr = K.dconv_bf16_weight_bytes(w.float(), bn).to(DEV)
    got = K.conv2d_direct(x.to(DEV), arr, (kh, kw), Cout, b.to(DEV), (s, s), pad, "relu", bn=bn,
                          maxpool_pad=mp, pool_rows=pool_rows).cpu()
    assert got.shape == ref.shape
    torch.testing.assert_close(got.float(), ref.float(), rtol=2e-2, atol=2e-2 * ref.abs().max().item())


FP8_POOL_CASES = [  # N, H, W, Cin, Cout, stride-1 3x3 pad, pool padding, bn
    (2, 37, 37, 32, 64, (0, 0, 0, 0), "VALID", 64),  # Inception Conv2d_2b -> MaxPool_3a at 1/4 scale
    (1, 30, 41, 32, 32, (1, 1, 1, 1), "SAME", 32),
    (2, 33, 33, 64, 64, (1, 1, 1, 1), "VALID", 64),
]


@pytest.mark.gpu
@pytest.mark.parametrize("pool_rows", [7, 14])
@pytest.mark.parametrize("case", FP8_POOL_CASES)
def test_dconv_fp8_maxpool_gpu(case, pool_rows):
    """fp8 -> fp8 direct conv + ReLU + fused 3x3/s2 max pool == the same kernel unpooled,
    then the fp8 pool kernel: bit-exact (the max runs over the same quantised bytes)."""
    N, H, W, Cin, Cout, pad, ppad, bn = case
    torch.manual_seed(H + Cin + Cout)
    x = torch.randn(N, H, W, Cin).relu()
    sx = Q.scale_for(x.max())
    xq = Q.quantize(x, sx).to(DEV)
    wq, ws = Q.quantize_weight(torch.randn(Cout, 3, 3, Cin) / (9 * Cin) ** 0.5)
    b = (torch.randn(Cout) * 0.1).to(DEV)
    arr = K.dconv_weights(wq, Cout, 1, bn).to(DEV)
    cs = (ws * sx).to(DEV)
    so = 0.02
    conv = K.conv2d_direct(xq, arr, (3, 3), Cout, b, (1, 1), pad, "relu", bn=bn, chan_scale=cs, out_scale=so)
    Ho, Wo = conv.shape[1:3]
    if ppad == "SAME":
        ph = max((-(-Ho // 2) - 1) * 2 + 3 - Ho, 0)
        pw = max((-(-Wo // 2) - 1) * 2 + 3 - Wo, 0)
        mp = (ph // 2, ph - ph // 2, pw // 2, pw - pw // 2)
    else:
        mp = (0, 0, 0, 0)
    ref = Q.pool2d_nhwc_fp8(conv, (3, 3), (2, 2), mp, "max").cpu()
    got = K.conv2d_direct(xq, arr, (3, 3), Cout, b, (1, 1), pad, "relu", bn=bn, chan_scale=cs, out_scale=so,
                          maxpool_pad=mp, pool_rows=pool_rows).cpu()
    assert got.shape == ref.shape and got.dtype == torch.uint8
    assert torch.equal(got, ref)
