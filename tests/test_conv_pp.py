"""``conv_pp`` (kernels/conv_pp.hip): implicit-GEMM NHWC convolution on the ping-pong MFMA
pipeline, checked against a plain PyTorch fp32 convolution of the same bf16 operands —
3x3 / 1x1 / strided / dilated / asymmetric (1x7, 7x1) filters, both tile shapes, M tails,
split-K, residual + ReLU epilogue, concat channel offsets and the dual-source (conv +
strided projection shortcut) mode."""
import pytest
import torch
import torch.nn.functional as F

from flink_tensorflow_amd.ops import kernels as K


def _ref(srcs, xs, w, bias, res, act, OH, OW):
    y = 0
    k0 = 0
    Cout = w.shape[0]
    for x, (sh, (KH, KW), (s_h, s_w), (pt, pl), (dh, dw)) in zip(xs, srcs):
        C = sh[3]
        wk = w[:, k0:k0 + KH * KW * C].float().reshape(Cout, KH, KW, C).permute(0, 3, 1, 2)
        k0 += KH * KW * C
        xi = F.pad(x.float().permute(0, 3, 1, 2), (pl, KW * dw, pt, KH * dh))
        y = y + F.conv2d(xi, wk, stride=(s_h, s_w), dilation=(dh, dw))[:, :, :OH, :OW]
    y = y.permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if act == "relu" else y


CASES = [
    # name, [(N,H,W,C), (KH,KW), stride, (pt,pl), dil], Cout, (OH, OW), residual, act
    # the 4-wave 128x128 LDS-DMA tile (conv_lite): 3x3 s1 / s2, N tail, M tail, residual,
    # dilation, 1xK / Kx1
    ("lite_3x3", [((4, 28, 28, 128), (3, 3), (1, 1), (1, 1), (1, 1))], 128, (28, 28), False, "relu"),
    ("lite_3x3s2", [((3, 28, 28, 256), (3, 3), (2, 2), (0, 0), (1, 1))], 256, (14, 14), False, "relu"),
    ("lite_tail", [((3, 7, 7, 512), (3, 3), (1, 1), (1, 1), (1, 1))], 200, (7, 7), True, "relu"),
    ("lite_tail_m", [((3, 7, 7, 512), (3, 3), (1, 1), (1, 1), (1, 1))], 512, (7, 7), False, None),
    ("lite_1x1", [((2, 14, 14, 256), (1, 1), (1, 1), (0, 0), (1, 1))], 1024, (14, 14), True, None),
    ("lite_dil", [((2, 17, 17, 64), (5, 5), (1, 1), (4, 4), (2, 2))], 192, (17, 17), False, "relu"),
    ("lite_1x7", [((2, 17, 17, 128), (1, 7), (1, 1), (0, 3), (1, 1))], 192, (17, 17), False, "relu"),
    ("lite_7x1", [((2, 17, 17, 192), (7, 1), (1, 1), (3, 0), (1, 1))], 136, (17, 17), False, None),
    # two sources on the 4-wave tile (expand + strided projection shortcut), M tail, N tail
    ("lite_dual", [((2, 14, 14, 128), (1, 1), (1, 1), (0, 0), (1, 1)),
                   ((2, 28, 28, 256), (1, 1), (2, 2), (0, 0), (1, 1))], 512, (14, 14), False, "relu"),
    ("lite_dual_s1", [((3, 7, 7, 64), (1, 1), (1, 1), (0, 0), (1, 1)),
                      ((3, 7, 7, 128), (1, 1), (1, 1), (0, 0), (1, 1))], 200, (7, 7), False, None),
]


def _run(case, dev, coff=0, tile=None):
    name, srcs, Cout, (OH, OW), with_res, act = case
    torch.manual_seed(0)
    xs = [torch.randn(s[0], device=dev).to(torch.bfloat16) for s in srcs]
    Ktot = sum(s[1][0] * s[1][1] * s[0][3] for s in srcs)
    w = (torch.randn(Cout, Ktot, device=dev) / Ktot ** 0.5).to(torch.bfloat16)
    bias = torch.randn(Cout, device=dev)
    N = srcs[0][0][0]
    res = torch.randn(N, OH, OW, Cout, device=dev).to(torch.bfloat16) if with_res else None
    cp = K.ConvPP(srcs, Cout, (OH, OW), dev, tile=tile)
    out = torch.zeros(N, OH, OW, Cout + coff, dtype=torch.bfloat16, device=dev)
    cp(xs, w, bias, res, act, out=out, out_channel_offset=coff)
    ref = _ref(srcs, xs, w, bias, res, act, OH, OW)
    return out[..., coff:].float(), ref, out[..., :coff]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv_pp_reference_host(case):
    got, ref, _ = _run(case, "cpu")
    torch.testing.assert_close(got, ref, atol=3e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv_pp_gpu(case):
    got, ref, _ = _run(case, "cuda")
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 2e-2 * scale + 2e-2, (case[0], err, scale)


@pytest.mark.gpu
def test_conv_pp_concat_offset_gpu():
    got, ref, left = _run(CASES[0], "cuda", coff=64)
    assert (got - ref).abs().max().item() <= 2e-2 * ref.abs().max().item() + 2e-2
    assert (left == 0).all()  # channels before the slice untouched


def test_removed_tiles_are_refused():
    with pytest.raises(ValueError):
        K.ConvPP([((2, 14, 14, 64), (3, 3), (1, 1), (1, 1), (1, 1))], 64, (14, 14), "cpu", tile=0)


def test_diagnostic_tiles_refuse_two_sources():
    with pytest.raises(ValueError):
        K.ConvPP([((2, 14, 14, 128), (1, 1), (1, 1), (0, 0), (1, 1)),
                  ((2, 28, 28, 256), (1, 1), (2, 2), (0, 0), (1, 1))], 512, (14, 14), "cpu", tile=4)
