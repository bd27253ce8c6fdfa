"""Neural-network op kernels with exact TF 1.x semantics (NHWC, SAME/VALID padding,
legacy ResizeBilinear coordinates, inference-mode FusedBatchNorm, LRN).

These are the semantic reference used by the interpreter and by CPU tests; the compiled
GPU plan (``graph/compiler.py``) lowers the same ops onto the hand-written CDNA4 kernels.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .op_registry import register


def same_pads(in_size: int, k: int, s: int, d: int = 1) -> tuple[int, int]:
    """TF SAME padding: (before, after), asymmetric with the extra pixel after."""
    eff = (k - 1) * d + 1
    out = math.ceil(in_size / s)
    total = max((out - 1) * s + eff - in_size, 0)
    return total // 2, total - total // 2


def conv_out_size(in_size: int, k: int, s: int, padding: str, d: int = 1, pads=(0, 0)) -> int:
    eff = (k - 1) * d + 1
    if padding == "SAME":
        return math.ceil(in_size / s)
    if padding == "VALID":
        return (in_size - eff) // s + 1
    return (in_size + pads[0] + pads[1] - eff) // s + 1


def _hw(attr, fmt):
    if attr is None:
        return 1, 1
    if len(attr) == 4:
        return (attr[1], attr[2]) if fmt == "NHWC" else (attr[2], attr[3])
    if len(attr) == 2:
        return attr[0], attr[1]
    return attr[0], attr[0]


def _explicit_pads(node, fmt):
    p = node.attr("explicit_paddings", []) or []
    if not p:
        return (0, 0), (0, 0)
    p = list(p)
    if fmt == "NHWC":
        return (p[2], p[3]), (p[4], p[5])
    return (p[4], p[5]), (p[6], p[7])


def conv2d_tf(x, w_hwio, strides=(1, 1), padding="SAME", dilations=(1, 1), explicit=((0, 0), (0, 0)), groups=1):
    """NHWC conv with TF padding semantics (torch reference)."""
    sh, sw = strides
    dh, dw = dilations
    kh, kw = w_hwio.shape[0], w_hwio.shape[1]
    xn = x.permute(0, 3, 1, 2)
    if padding == "SAME":
        ph = same_pads(x.shape[1], kh, sh, dh)
        pw = same_pads(x.shape[2], kw, sw, dw)
    elif padding == "VALID":
        ph, pw = (0, 0), (0, 0)
    else:
        ph, pw = explicit
    if any(ph) or any(pw):
        xn = F.pad(xn, (pw[0], pw[1], ph[0], ph[1]))
    w = w_hwio.permute(3, 2, 0, 1)  # OIHW
    y = F.conv2d(xn, w.to(xn.dtype), stride=(sh, sw), dilation=(dh, dw), groups=groups)
    return y.permute(0, 2, 3, 1).contiguous()


@register("Conv2D")
def _conv2d(ctx, node, x, w):
    fmt = node.attr("data_format", "NHWC")
    s = _hw(node.attr("strides"), fmt)
    d = _hw(node.attr("dilations"), fmt)
    pad = node.attr("padding", "SAME")
    if fmt == "NCHW":
        x = x.permute(0, 2, 3, 1)
    y = conv2d_tf(x, w, s, pad, d, _explicit_pads(node, fmt))
    if fmt == "NCHW":
        y = y.permute(0, 3, 1, 2).contiguous()
    return (y,)


@register("DepthwiseConv2dNative")
def _dwconv(ctx, node, x, w):
    fmt = node.attr("data_format", "NHWC")
    s = _hw(node.attr("strides"), fmt)
    d = _hw(node.attr("dilations"), fmt)
    kh, kw, cin, mult = w.shape
    w2 = w.reshape(kh, kw, 1, cin * mult)
    return (conv2d_tf(x, w2, s, node.attr("padding", "SAME"), d, groups=cin),)


def pool_tf(x, ksize, strides, padding, mode):
    kh, kw = ksize
    sh, sw = strides
    xn = x.permute(0, 3, 1, 2)
    if padding == "SAME":
        ph = same_pads(x.shape[1], kh, sh)
        pw = same_pads(x.shape[2], kw, sw)
    else:
        ph, pw = (0, 0), (0, 0)
    if mode == "max":
        if any(ph) or any(pw):
            xn = F.pad(xn, (pw[0], pw[1], ph[0], ph[1]), value=float("-inf"))
        y = F.max_pool2d(xn, (kh, kw), (sh, sw))
    else:
        # TF AvgPool SAME excludes padding from the divisor
        if any(ph) or any(pw):
            xp = F.pad(xn, (pw[0], pw[1], ph[0], ph[1]))
            ones = F.pad(torch.ones_like(xn[:, :1]), (pw[0], pw[1], ph[0], ph[1]))
            ssum = F.avg_pool2d(xp, (kh, kw), (sh, sw), divisor_override=1)
            cnt = F.avg_pool2d(ones, (kh, kw), (sh, sw), divisor_override=1)
            y = ssum / cnt
        else:
            y = F.avg_pool2d(xn, (kh, kw), (sh, sw))
    return y.permute(0, 2, 3, 1).contiguous()


@register("MaxPool", "MaxPoolV2")
def _maxpool(ctx, node, x, *rest):
    fmt = node.attr("data_format", "NHWC")
    k = _hw(node.attr("ksize"), fmt)
    s = _hw(node.attr("strides"), fmt)
    return (pool_tf(x, k, s, node.attr("padding", "VALID"), "max"),)


@register("AvgPool")
def _avgpool(ctx, node, x):
    fmt = node.attr("data_format", "NHWC")
    k = _hw(node.attr("ksize"), fmt)
    s = _hw(node.attr("strides"), fmt)
    return (pool_tf(x, k, s, node.attr("padding", "VALID"), "avg"),)


def fused_batch_norm_inference(x, scale, offset, mean, var, eps):
    inv = torch.rsqrt(var.float() + eps) * scale.float()
    return (x.float() * inv + (offset.float() - mean.float() * inv)).to(x.dtype)


@register("FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3")
def _fused_bn(ctx, node, x, scale, offset, mean, var):
    eps = node.attr("epsilon", 1e-3)
    fmt = node.attr("data_format", "NHWC")
    if node.attr("is_training", True) and mean.numel() == 0:
        dims = (0, 1, 2) if fmt == "NHWC" else (0, 2, 3)
        mean = x.float().mean(dims)
        var = x.float().var(dims, unbiased=False)
    if fmt == "NCHW":
        sh = (1, -1, 1, 1)
        y = (x - mean.reshape(sh)) * torch.rsqrt(var.reshape(sh) + eps) * scale.reshape(sh) + offset.reshape(sh)
    else:
        y = fused_batch_norm_inference(x, scale, offset, mean, var, eps)
    z = torch.zeros(0, device=x.device)
    return (y, mean, var, z, z, z)


@register("LRN")
def _lrn(ctx, node, x):
    r = node.attr("depth_radius", 5)
    bias = node.attr("bias", 1.0)
    alpha = node.attr("alpha", 1.0)
    beta = node.attr("beta", 0.5)
    sq = (x.float() ** 2).permute(0, 3, 1, 2)  # N C H W
    c = sq.shape[1]
    pad = F.pad(sq, (0, 0, 0, 0, r, r))
    acc = torch.zeros_like(sq)
    for i in range(2 * r + 1):
        acc = acc + pad[:, i:i + c]
    y = x.float() / (bias + alpha * acc.permute(0, 2, 3, 1)) ** beta
    return (y.to(x.dtype),)


def resize_bilinear_tf(x, oh, ow, align_corners=False, half_pixel_centers=False):
    """TF ResizeBilinear on NHWC (float math; legacy coordinates by default)."""
    n, ih, iw, c = x.shape
    dev = x.device

    def scale(i, o):
        if align_corners and o > 1:
            return (i - 1) / (o - 1)
        return i / o

    sy, sx = scale(ih, oh), scale(iw, ow)
    ys = torch.arange(oh, device=dev, dtype=torch.float32)
    xs = torch.arange(ow, device=dev, dtype=torch.float32)
    if half_pixel_centers:
        fy = (ys + 0.5) * sy - 0.5
        fx = (xs + 0.5) * sx - 0.5
    else:
        fy = ys * sy
        fx = xs * sx
    y0 = torch.clamp(torch.floor(fy), min=0).long()
    x0 = torch.clamp(torch.floor(fx), min=0).long()
    y1 = torch.clamp(y0 + 1, max=ih - 1)
    x1 = torch.clamp(x0 + 1, max=iw - 1)
    wy = (fy - torch.floor(fy)).clamp(0, 1) if not half_pixel_centers else (fy - y0.float()).clamp(0, 1)
    wx = (fx - torch.floor(fx)).clamp(0, 1) if not half_pixel_centers else (fx - x0.float()).clamp(0, 1)
    xf = x.float()
    top = xf[:, y0][:, :, x0] * (1 - wx)[None, None, :, None] + xf[:, y0][:, :, x1] * wx[None, None, :, None]
    bot = xf[:, y1][:, :, x0] * (1 - wx)[None, None, :, None] + xf[:, y1][:, :, x1] * wx[None, None, :, None]
    return top * (1 - wy)[None, :, None, None] + bot * wy[None, :, None, None]


@register("ResizeBilinear")
def _resize_bilinear(ctx, node, x, size):
    oh, ow = [int(v) for v in size.reshape(-1).tolist()]
    return (resize_bilinear_tf(x, oh, ow, node.attr("align_corners", False), node.attr("half_pixel_centers", False)),)


@register("ResizeNearestNeighbor")
def _resize_nn(ctx, node, x, size):
    oh, ow = [int(v) for v in size.reshape(-1).tolist()]
    n, ih, iw, c = x.shape
    ys = torch.clamp((torch.arange(oh, device=x.device) * (ih / oh)).floor().long(), max=ih - 1)
    xs = torch.clamp((torch.arange(ow, device=x.device) * (iw / ow)).floor().long(), max=iw - 1)
    return (x[:, ys][:, :, xs],)


@register("L2Normalize")
def _l2n(ctx, node, x):
    return (F.normalize(x, dim=-1),)
