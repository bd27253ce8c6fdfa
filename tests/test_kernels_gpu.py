"""Numerics of the hand-written CDNA4 kernels vs plain PyTorch fp32 references.

Inputs are generated in bf16 on the host; the reference runs the same bf16 values in
fp32 on the CPU (``ops.kernels`` host path), the kernel runs on the GPU.  Tolerances are
set by bf16 output rounding (8 significant bits) and fp32 accumulation-order noise.
"""
import pytest
import torch

from flink_tensorflow_amd.ops import kernels as K

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _close(got, ref, rtol=2e-2, atol_scale=2e-2):
    got = got.float().cpu()
    ref = ref.float().cpu()
    atol = atol_scale * max(ref.abs().max().item(), 1e-3)
    torch.testing.assert_close(got, ref, rtol=rtol, atol=atol)


CONV_CASES = [
    # N, H, W, Cin, Cout, K, stride, pad(t,b,l,r), act, residual, bias
    (2, 56, 56, 64, 64, 1, 1, (0, 0, 0, 0), "relu", False, True),
    (2, 56, 56, 64, 256, 1, 1, (0, 0, 0, 0), "none", True, True),
    (2, 28, 28, 128, 128, 3, 1, (1, 1, 1, 1), "relu", False, True),
    (2, 56, 56, 128, 128, 3, 2, (0, 1, 0, 1), "relu", False, True),
    (2, 224, 224, 8, 64, 7, 2, (2, 3, 2, 3), "relu", False, True),
    (3, 7, 7, 512, 2048, 1, 1, (0, 0, 0, 0), "relu", True, True),
    (1, 14, 14, 256, 1000, 1, 1, (0, 0, 0, 0), "none", False, False),  # Cout tail
    (2, 17, 17, 192, 160, 1, 7, (0, 0, 0, 0), "relu", False, True),
    (2, 9, 11, 64, 96, 3, 1, (1, 1, 1, 1), "relu6", False, True),       # M tail
]


@pytest.mark.parametrize("cfg", [-1])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_nhwc(case, cfg):
    """cfg -1: auto register-staged tiles."""
    N, H, W, Cin, Cout, k, s, pad, act, has_res, has_b = case
    kh, kw = (k, k) if k != 7 or Cin == 8 else (1, 7)
    if case[5] == 1 and case[6] == 7:  # the 1x7 Inception-style case
        kh, kw, s = 1, 7, 1
        pad = (0, 0, 3, 3)
    g = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(N, H, W, Cin, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, kh, kw, Cin, generator=g) / (kh * kw * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g) if has_b else None
    Ho, Wo = K.conv_out_hw(H, W, kh, kw, s, s, pad[0], pad[2], 1, 1, pad[1], pad[3])
    r = torch.randn(N, Ho, Wo, Cout, generator=g).to(torch.bfloat16) if has_res else None
    ref = K.conv2d_nhwc(x, w, b, r, (s, s), pad, (1, 1), act)
    got = K.conv2d_nhwc(x.to(DEV), w.to(DEV), b.to(DEV) if b is not None else None,
                        r.to(DEV) if r is not None else None, (s, s), pad, (1, 1), act, cfg=cfg)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    _close(got, ref)


def test_conv_identity_asymmetric():
    """A = I check with an asymmetric B (guide §3): catches a transposed C-write."""
    N, H, W, C = 1, 4, 4, 64
    x = torch.arange(N * H * W * C, dtype=torch.float32).reshape(N, H, W, C).remainder(7).to(torch.bfloat16)
    w = torch.eye(C).reshape(C, 1, 1, C).to(torch.bfloat16)
    got = K.conv2d_nhwc(x.to(DEV), w.to(DEV))
    assert torch.equal(got.cpu(), x)


@pytest.mark.parametrize("cfg", [-1])
def test_conv_concat_slice_write(cfg):
    x = torch.randn(2, 8, 8, 64).to(torch.bfloat16).to(DEV)
    w1 = torch.randn(32, 1, 1, 64).to(torch.bfloat16).to(DEV)
    w2 = torch.randn(64, 1, 1, 64).to(torch.bfloat16).to(DEV)
    out = torch.zeros(2, 8, 8, 96, dtype=torch.bfloat16, device=DEV)
    K.conv2d_nhwc(x, w1, out=out, out_channel_offset=0, cfg=cfg)
    K.conv2d_nhwc(x, w2, out=out, out_channel_offset=32, cfg=cfg)
    ref = torch.cat([K.conv2d_nhwc(x, w1), K.conv2d_nhwc(x, w2)], -1)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("M,N,Kd,act", [(256, 1000, 2048, "none"), (77, 3072, 768, "gelu"), (5, 64, 64, "relu"),
                                         (1024, 768, 3072, "none")])
def test_gemm(M, N, Kd, act):
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, Kd, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, Kd, generator=g) / Kd ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, generator=g)
    ref = K.gemm(x, w, b, None, act)
    got = K.gemm(x.to(DEV), w.to(DEV), b.to(DEV), None, act)
    _close(got, ref)


@pytest.mark.parametrize("hw_in,hw_out,half", [((256, 256), (224, 224), False), ((224, 224), (224, 224), False),
                                               ((300, 200), (224, 224), True)])
def test_preprocess(hw_in, hw_out, half):
    img = torch.randint(0, 256, (3, *hw_in, 3), dtype=torch.uint8)
    mean, std = (123.68, 116.78, 103.94), (58.4, 57.12, 57.38)
    ref = K.preprocess_images(img, hw_out, mean, std, False, half)
    got = K.preprocess_images(img.to(DEV), hw_out, mean, std, False, half)
    _close(got, ref, rtol=1e-2, atol_scale=1e-2)
    assert (got[..., 3:] == 0).all()


@pytest.mark.parametrize("hw_in,hw_out,half,align", [((256, 256), (224, 224), False, False),
                                                     ((100, 120), (75, 75), False, False),  # odd: zero-filled edge
                                                     ((320, 300), (299, 299), True, False),
                                                     ((299, 299), (299, 299), False, False),  # 897-B rows
                                                     ((64, 96), (33, 47), False, True),
                                                     ((400, 480), (224, 224), False, False)])  # 4 KiB rows
def test_preprocess_s2d_row_staged(hw_in, hw_out, half, align):
    """The row-staged (LDS) s2d preprocess kernel vs the fp32 host path."""
    img = torch.randint(0, 256, (4, *hw_in, 3), dtype=torch.uint8)
    mean, std = (123.68, 116.78, 103.94), (58.4, 57.12, 57.38)
    got = K.preprocess_images(img.to(DEV), hw_out, mean, std, align, half, s2d=True)
    ref = K.preprocess_images(img, hw_out, mean, std, align, half, s2d=True)
    _close(got, ref, rtol=1e-2, atol_scale=1e-2)
    assert (got[..., 12:] == 0).all()


@pytest.mark.parametrize("mode,k,s,pad", [("max", 3, 2, (0, 1, 0, 1)), ("avg", 3, 1, (1, 1, 1, 1)),
                                          ("max", 2, 2, (0, 0, 0, 0)), ("avg", 8, 8, (0, 0, 0, 0))])
def test_pool(mode, k, s, pad):
    x = torch.randn(2, 16, 16, 64).to(torch.bfloat16)
    ref = K.pool2d_nhwc(x, (k, k), (s, s), pad, mode)
    got = K.pool2d_nhwc(x.to(DEV), (k, k), (s, s), pad, mode)
    _close(got, ref, rtol=1e-2, atol_scale=1e-2)


def test_global_avgpool():
    x = torch.randn(4, 7, 7, 2048).to(torch.bfloat16)
    _close(K.global_avgpool(x.to(DEV)), K.global_avgpool(x), rtol=1e-2, atol_scale=1e-2)


@pytest.mark.parametrize("C,k", [(1000, 5), (10, 3), (4096, 1)])
def test_softmax_topk(C, k):
    logits = (torch.randn(37, C) * 3).to(torch.bfloat16)
    v_ref, i_ref, p_ref = K.softmax_topk(logits, k, want_probs=True)
    v, i, p = K.softmax_topk(logits.to(DEV), k, want_probs=True)
    _close(p, p_ref, rtol=1e-2, atol_scale=1e-2)
    torch.testing.assert_close(v.cpu(), v_ref, rtol=1e-3, atol=1e-4)
    # indices: equal except where probabilities tie in bf16
    mism = (i.cpu() != i_ref)
    if mism.any():
        pf = torch.softmax(logits.float(), -1)
        assert torch.allclose(pf.gather(1, i.cpu().long()), v_ref, atol=1e-3)


@pytest.mark.parametrize("D", [768, 1024, 64])
def test_layernorm(D):
    x = torch.randn(33, D).to(torch.bfloat16)
    r = torch.randn(33, D).to(torch.bfloat16)
    gm, bt = torch.randn(D), torch.randn(D)
    ref = K.layernorm(x, gm, bt, r)
    got = K.layernorm(x.to(DEV), gm.to(DEV), bt.to(DEV), r.to(DEV))
    _close(got, ref)


def test_linear_autograd():
    from flink_tensorflow_amd.ops.autograd import linear

    x = torch.randn(64, 96).to(torch.bfloat16)
    w = (torch.randn(32, 96) / 10).to(torch.bfloat16)
    b = torch.randn(32)
    xs = [x.clone().requires_grad_(True), x.to(DEV).requires_grad_(True)]
    ws = [w.clone().float().requires_grad_(True), w.to(DEV).requires_grad_(True)]
    bs = [b.clone().requires_grad_(True), b.to(DEV).requires_grad_(True)]
    outs = []
    for i in range(2):
        y = linear(xs[i], ws[i] if i else ws[i].to(torch.bfloat16), bs[i], "relu")
        y.float().sum().backward()
        outs.append(y)
    _close(outs[1], outs[0])
    _close(xs[1].grad, xs[0].grad)
    _close(bs[1].grad, bs[0].grad)
    # fp32 master weight + bf16 compute copy (ops.autograd.Linear on the GPU): the fp32
    # gradient lands on the master straight from the library GEMM
    wm = w.to(DEV).float().requires_grad_(True)
    x3 = x.to(DEV).requires_grad_(True)
    y = linear(x3, wm, bs[1].detach(), "relu", w_compute=wm.detach().to(torch.bfloat16))
    y.float().sum().backward()
    assert wm.grad.dtype == torch.float32
    _close(wm.grad, ws[0].grad)


@pytest.mark.parametrize("hw", [224, 299, 100])
def test_preprocess_s2d(hw):
    img = torch.randint(0, 256, (3, 256, 256, 3), dtype=torch.uint8)
    ref = K.preprocess_images(img, (hw, hw), s2d=True)
    got = K.preprocess_images(img.to(DEV), (hw, hw), s2d=True)
    _close(got, ref, rtol=1e-2, atol_scale=1e-2)


@pytest.mark.parametrize("stride2,cfg", [(1, -1), (2, -1), (2, 0), (1, 3)])
def test_conv1x1_dual(stride2, cfg):
    """Expansion conv + fused (strided) projection shortcut vs the two-conv reference."""
    g = torch.Generator().manual_seed(11 + stride2)
    N, Ho, Wo, K1, C2, Cout = 2, 14, 14, 64, 96, 256
    x = torch.randn(N, Ho, Wo, K1, generator=g).to(torch.bfloat16)
    x2 = torch.randn(N, Ho * stride2, Wo * stride2, C2, generator=g).to(torch.bfloat16)
    w = (torch.randn(Cout, K1 + C2, generator=g) / 12).to(torch.bfloat16)
    b = torch.randn(Cout, generator=g)
    ref = K.conv1x1_dual(x, x2, w, b, stride2, "relu")
    two = K.conv2d_nhwc(x, w[:, :K1].reshape(Cout, 1, 1, K1), b,
                        K.conv2d_nhwc(x2, w[:, K1:].reshape(Cout, 1, 1, C2), None, None, (stride2, stride2)),
                        act="relu")
    torch.testing.assert_close(ref, two, rtol=1e-2, atol=1e-2)
    got = K.conv1x1_dual(x.to(DEV), x2.to(DEV), w.to(DEV), b.to(DEV), stride2, "relu", cfg=cfg)
    _close(got, ref)


@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "max", "rsub"])
def test_binary_elementwise(op):
    g = torch.Generator().manual_seed(3)
    a = torch.randn(3, 5, 64, generator=g).to(torch.bfloat16)
    b_full = (torch.rand(3, 5, 64, generator=g) + 0.5).to(torch.bfloat16)
    b_vec = torch.rand(64, generator=g) + 0.5
    for b in (b_full, b_vec, 1.5):
        ref = K.binary(a, b, op, act="relu")
        got = K.binary(a.to(DEV), b.to(DEV) if torch.is_tensor(b) else b, op, act="relu")
        _close(got, ref)


def test_lrn_kernel():
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 7, 7, 96, generator=g).to(torch.bfloat16)
    ref = K.lrn(x, 5, 1.0, 1e-2, 0.75)
    got = K.lrn(x.to(DEV), 5, 1.0, 1e-2, 0.75)
    _close(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 56, 56), (3, 20, 40), (1, 8, 32), (2, 13, 37)])
@pytest.mark.parametrize("act", [None, "relu"])
def test_conv3x3_c64_kernel(shape, act):
    """Persistent LDS-resident-weights 3x3 conv vs the fp32 reference (edge tiles overlap
    when H % 8 or W % 32 != 0; output written into a wider buffer at a channel offset)."""
    from flink_tensorflow_amd.ops import kernels as K

    N, H, W = shape
    g = torch.Generator().manual_seed(H * W)
    x = torch.randn(N, H, W, 64, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, 3, 3, 64, generator=g) * 0.05).to(torch.bfloat16)
    b = torch.randn(64, generator=g)
    ref = K.conv2d_nhwc(x.float(), w.float(), b, None, (1, 1), (1, 1, 1, 1), (1, 1), act)
    out = torch.full((N, H, W, 96), 7.0, dtype=torch.bfloat16, device="cuda")
    K.conv3x3_c64(x.cuda(), w.cuda(), b.cuda(), act, out=out, out_channel_offset=16)
    torch.cuda.synchronize()
    got = out[..., 16:80].float().cpu()
    torch.testing.assert_close(got, ref, rtol=2e-2, atol=3e-2)
    assert (out[..., :16] == 7).all() and (out[..., 80:] == 7).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cn", [64, 128])
@pytest.mark.parametrize("M", [2 * 56 * 56, 1000 + 37, 50])
def test_bottleneck_tail_kernel(cn, M):
    """Fused 1x1 expand (+residual, ReLU) -> 1x1 reduce (+ReLU) vs the two fp32 reference
    convs; M not a multiple of the pixel tile exercises the tail tile, M < tile a single
    partial tile."""
    g = torch.Generator().manual_seed(M + cn)
    x2 = torch.randn(M, 64, generator=g).to(torch.bfloat16)
    res = torch.randn(M, 256, generator=g).to(torch.bfloat16)
    w3 = (torch.randn(256, 64, generator=g) * 0.1).to(torch.bfloat16)
    w1 = (torch.randn(cn, 256, generator=g) * 0.05).to(torch.bfloat16)
    b3, b1 = torch.randn(256, generator=g), torch.randn(cn, generator=g)
    y3_ref = torch.relu(x2.float() @ w3.float().t() + b3 + res.float())
    y1_ref = torch.relu(y3_ref.to(torch.bfloat16).float() @ w1.float().t() + b1)
    y3, y1 = K.bottleneck_tail(x2.to(DEV), res.to(DEV), w3.to(DEV), b3.to(DEV), w1.to(DEV), b1.to(DEV))
    torch.cuda.synchronize()
    _close(y3, y3_ref)
    _close(y1, y1_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [2 * 56 * 56, 1000 + 37])
def test_bottleneck_tail_dual_kernel(M):
    """Dual form: [x2 | xs] . [W3 | Wsc]^T (expand + stride-1 projection shortcut) -> relu
    -> 1x1 reduce, vs the fp32 reference."""
    g = torch.Generator().manual_seed(M)
    x2 = torch.randn(M, 64, generator=g).to(torch.bfloat16)
    xs = torch.randn(M, 64, generator=g).to(torch.bfloat16)
    w3 = (torch.randn(256, 128, generator=g) * 0.1).to(torch.bfloat16)
    w1 = (torch.randn(64, 256, generator=g) * 0.05).to(torch.bfloat16)
    b3, b1 = torch.randn(256, generator=g), torch.randn(64, generator=g)
    y3_ref = torch.relu(torch.cat([x2, xs], 1).float() @ w3.float().t() + b3)
    y1_ref = torch.relu(y3_ref.to(torch.bfloat16).float() @ w1.float().t() + b1)
    y3, y1 = K.bottleneck_tail(x2.to(DEV), None, w3.to(DEV), b3.to(DEV), w1.to(DEV), b1.to(DEV), xs=xs.to(DEV))
    torch.cuda.synchronize()
    _close(y3, y3_ref)
    _close(y1, y1_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("D,dtype", [(768, torch.bfloat16), (64, torch.float32)])
def test_gather_rows_kernel(D, dtype):
    """First-token (CLS) row gather of the packed encoder: == torch indexing; an index
    out of range gives a zero row."""
    from flink_tensorflow_amd.ops import kernels as K

    dev = torch.device("cuda", 0)
    x = torch.randn(1000, D, device=dev).to(dtype)
    idx = torch.tensor([0, 999, 5, 5, -1, 1000, 17], dtype=torch.int32, device=dev)
    got = K.gather_rows(x, idx)
    want = torch.zeros_like(got)
    ok = (idx >= 0) & (idx < 1000)
    want[ok] = x[idx[ok].long()]
    assert torch.equal(got, want)
