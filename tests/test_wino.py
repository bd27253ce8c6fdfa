"""Winograd F(2x2, 3x3) conv (kernels/wino3x3.hip): the algebra and the weight-fragment
layout on the host, the kernel against a plain fp32 conv on the GPU."""
import pytest
import torch
import torch.nn.functional as F

from flink_tensorflow_amd.ops import kernels as K


def _ref_conv(x_nhwc, w_hwio, bias, relu):
    y = F.conv2d(x_nhwc.permute(0, 3, 1, 2).float(), w_hwio.permute(3, 2, 0, 1).float(), bias.float(), padding=1)
    y = y.permute(0, 2, 3, 1)
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("N,H,W,C,Co", [(2, 8, 8, 32, 64), (1, 7, 7, 64, 64), (3, 5, 9, 32, 128), (2, 14, 14, 64, 64)])
def test_wino_algebra_matches_conv(N, H, W, C, Co):
    g = torch.Generator().manual_seed(N * H + C)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(3, 3, C, Co, generator=g) * 0.1
    b = torch.randn(Co, generator=g)
    u = K.wino_f23_weights(w)
    assert u.dtype == torch.float16 and u.numel() == 16 * C * Co
    ref = _ref_conv(x, w, b, True)
    exact = K.wino_f23_reference(x, u, Co, b, K.ACT_RELU, fp16_domain=False)
    # only U's fp16 rounding separates the two
    assert (exact - ref).abs().max() <= 2e-3 * ref.abs().max()
    f16 = K.wino_f23_reference(x, u, Co, b, K.ACT_RELU, fp16_domain=True)
    assert (f16 - ref).abs().max() <= 4e-3 * ref.abs().max()
    # host path of the op
    out = K.wino_f23(x, u, Co, b, K.ACT_RELU)
    assert torch.allclose(out, exact, atol=1e-5, rtol=0)


def test_wino_fragment_layout():
    """Lane r + 32 h of fragment (cbg, ks, xi) holds U[xi][16 ks + 8 h + j][32 cbg + r]."""
    C, Co = 32, 64
    w = torch.randn(3, 3, C, Co)
    u = K.wino_f23_weights(w).reshape(Co // 32, C // 16, 16, 64, 8).float()
    G = torch.tensor(K._WG, dtype=torch.float64)
    U = torch.einsum("ia,abck,jb->ijck", G, w.double(), G).reshape(16, C, Co).half().float()
    for cbg, ks, xi, lane, j in [(0, 0, 0, 0, 0), (1, 1, 5, 37, 3), (0, 1, 15, 63, 7), (1, 0, 9, 31, 6)]:
        r, h = lane & 31, lane >> 5
        assert u[cbg, ks, xi, lane, j] == U[xi, 16 * ks + 8 * h + j, 32 * cbg + r]


def test_wino_eligibility():
    assert K.wino_f23_eligible((256, 56, 56, 64), (64, 3, 3, 64), (1, 1), (1, 1, 1, 1), (1, 1), None, K.ACT_RELU)
    assert K.wino_f23_eligible((256, 7, 7, 512), (512, 3, 3, 512), (1, 1), (1, 1, 1, 1), (1, 1), None, K.ACT_RELU)
    assert not K.wino_f23_eligible((8, 56, 56, 64), (64, 3, 3, 64), (2, 2), (1, 1, 1, 1), (1, 1), None, K.ACT_RELU)
    assert not K.wino_f23_eligible((8, 56, 56, 48), (64, 3, 3, 48), (1, 1), (1, 1, 1, 1), (1, 1), None, K.ACT_RELU)
    assert not K.wino_f23_eligible((8, 56, 56, 64), (96, 3, 3, 64), (1, 1), (1, 1, 1, 1), (1, 1), None, K.ACT_RELU)
    # a 64-tile block of a 224-wide image stages more than the kernel's per-thread budget
    assert not K.wino_f23_eligible((2, 224, 224, 64), (64, 3, 3, 64), (1, 1), (1, 1, 1, 1), (1, 1), None, None)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,W,C,Co,relu,coff", [
    (4, 56, 56, 64, 64, True, 0),
    (3, 28, 28, 128, 128, True, 0),
    (5, 14, 14, 256, 256, True, 0),
    (6, 7, 7, 512, 512, True, 0),
    (2, 9, 13, 96, 192, False, 64),
    (1, 3, 3, 32, 64, True, 0),
])
def test_wino_kernel_vs_fp32(N, H, W, C, Co, relu, coff):
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(H * W + C)
    x = torch.randn(N, H, W, C, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(3, 3, C, Co, generator=g) * (2.0 / (9 * C)) ** 0.5
    b = (torch.randn(Co, generator=g) * 0.1).to(dev)
    u = K.wino_f23_weights(w).to(dev)
    out = torch.full((N, H, W, Co + coff + 8), 7.0, dtype=torch.bfloat16, device=dev)
    K.wino_f23(x, u, Co, b, K.ACT_RELU if relu else K.ACT_NONE, out=out, out_channel_offset=coff)
    torch.cuda.synchronize()
    ref = _ref_conv(x.float().cpu(), w, b.cpu(), relu)
    got = out[..., coff:coff + Co].float().cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1.5e-2 * scale, (err, scale)
    # the channels outside [coff, coff + Co) are untouched
    assert (out[..., :coff] == 7.0).all() and (out[..., coff + Co:] == 7.0).all()
