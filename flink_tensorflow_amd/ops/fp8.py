"""OCP FP8 (e4m3fn) ops: weight/activation quantisation and the fp8 MFMA conv/GEMM,
pooling and global-average-pool kernels of ``kernels/fp8.hip``.

fp8 tensors are carried as raw ``torch.uint8`` storage (one e4m3fn byte per element) plus
a float scale: ``value = e4m3(byte) * scale``.  Weights have one scale per output
channel, activations one scale per buffer (static, calibrated by the graph compiler).
On host tensors every op runs an fp32 reference with identical quantisation points
(dequantise → fp32 op → saturate/round to e4m3), which the GPU tests compare against.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .kernels import _apply_act_ref, _check, _hip, _stream, act_code, conv_out_hw

FP8_MAX = 448.0
E4M3 = torch.float8_e4m3fn


def to_fp8_bytes(x: torch.Tensor) -> torch.Tensor:
    """float tensor (already divided by its scale) → uint8 e4m3fn bytes (RNE, saturating)."""
    return x.float().clamp(-FP8_MAX, FP8_MAX).to(E4M3).view(torch.uint8)


def from_fp8_bytes(b: torch.Tensor) -> torch.Tensor:
    return b.view(E4M3).float()


def scale_for(amax: float, margin: float = 1.0) -> float:
    """Per-tensor scale mapping ``amax`` onto the e4m3 range (guarding all-zero tensors)."""
    amax = float(amax) * margin
    return amax / FP8_MAX if amax > 0 else 1.0


def quantize_weight(w: torch.Tensor):
    """``w`` [Cout, ...] float → (uint8 [Cout, K] e4m3 bytes, fp32 per-channel scales [Cout])."""
    w2 = w.detach().float().reshape(w.shape[0], -1)
    amax = w2.abs().amax(1)
    scale = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    return to_fp8_bytes(w2 / scale[:, None]).contiguous(), scale.contiguous()


def quantize(x: torch.Tensor, scale: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """bf16/float → fp8 bytes with ``x / scale``."""
    if x.is_cuda:
        _check(x, "x", torch.bfloat16, x.device)
        if out is None:
            out = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        _hip().quantize_bf16_fp8(x.data_ptr(), out.data_ptr(), x.numel(), 1.0 / scale, _stream())
        return out
    q = to_fp8_bytes(x.float() / scale)
    if out is not None:
        out.copy_(q)
        return out
    return q


def dequantize(q: torch.Tensor, scale: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """fp8 bytes → bf16 (device) / fp32 (host) ``q * scale``."""
    if q.is_cuda:
        if out is None:
            out = torch.empty(q.shape, dtype=torch.bfloat16, device=q.device)
        _hip().dequantize_fp8_bf16(q.data_ptr(), out.data_ptr(), q.numel(), float(scale), _stream())
        return out
    y = from_fp8_bytes(q) * scale
    if out is not None:
        out.copy_(y)
        return out
    return y


def conv2d_nhwc_fp8(x: torch.Tensor, x_scale: float, wq: torch.Tensor, kshape, w_scale: torch.Tensor,
                    bias: torch.Tensor | None = None, stride=(1, 1), pad=(0, 0, 0, 0), dilation=(1, 1), act=None,
                    out_scale: float | None = None, out: torch.Tensor | None = None, out_channel_offset: int = 0,
                    cfg: int = -1, chan_scale: torch.Tensor | None = None) -> torch.Tensor:
    """fp8 implicit-GEMM Conv2D.

    ``x``: NHWC fp8 bytes (uint8) with scale ``x_scale``, or bf16 (quantised on load by
    ``1/x_scale``).  ``wq`` [Cout, KH*KW*Cin] e4m3 bytes with ``kshape = (KH, KW)`` and
    per-channel ``w_scale``.  ``out_scale`` = None → bf16 output, else fp8 bytes with that
    scale.  ``pad`` = (top, bottom, left, right); ``out`` may be a wider NHWC buffer
    (concat target) written at ``out_channel_offset``.  ``chan_scale`` = precomputed
    ``w_scale * x_scale`` (the compiled plan passes it to stay allocation-free).
    """
    N, H, W, Cin = x.shape
    Cout = wq.shape[0]
    KH, KW = kshape
    sh, sw = stride
    pt, pb, pl, pr = pad
    dh, dw = dilation
    Ho, Wo = conv_out_hw(H, W, KH, KW, sh, sw, pt, pl, dh, dw, pb, pr)
    a = act_code(act)
    out_fp8 = out_scale is not None
    odt = torch.uint8 if out_fp8 else (torch.bfloat16 if x.is_cuda else torch.float32)
    if out is None:
        out = torch.empty((N, Ho, Wo, Cout), dtype=odt, device=x.device)
        out_channel_offset = 0
    if out.shape[:3] != (N, Ho, Wo) or out_channel_offset + Cout > out.shape[3]:
        raise ValueError(f"conv2d_nhwc_fp8: out {tuple(out.shape)} cannot hold [{N},{Ho},{Wo},{Cout}] at "
                         f"offset {out_channel_offset}")
    ldy = out.shape[-1]
    if x.is_cuda:
        in_bf16 = x.dtype == torch.bfloat16
        if not in_bf16:
            _check(x, "x", torch.uint8, x.device)
        _check(wq, "wq", torch.uint8, x.device)
        if wq.shape[1] != KH * KW * Cin:
            raise ValueError(f"conv2d_nhwc_fp8: weight K {wq.shape[1]} != {KH}*{KW}*{Cin}")
        if chan_scale is None:
            chan_scale = (w_scale.float() * x_scale).contiguous()
        if bias is None:
            from .kernels import _zeros_bias

            bias = _zeros_bias(Cout, x.device)
        _check(chan_scale, "chan_scale", torch.float32, x.device)
        _check(bias, "bias", torch.float32, x.device)
        _check(out, "out", odt, x.device)
        _hip().conv2d_nhwc_fp8(x.data_ptr(), wq.data_ptr(), chan_scale.data_ptr(), bias.data_ptr(), out.data_ptr(), N,
                               H, W, Cin, Cout, KH, KW, sh, sw, pt, pl, dh, dw, Ho, Wo, ldy, out_channel_offset,
                               int(in_bf16), 1.0 / x_scale, int(out_fp8), 1.0 / out_scale if out_fp8 else 1.0, a,
                               _stream(), cfg)
        return out
    # host reference with the same quantisation points
    if x.dtype == torch.uint8:
        xf = from_fp8_bytes(x) * x_scale
    else:
        xf = from_fp8_bytes(to_fp8_bytes(x.float() / x_scale)) * x_scale
    wf = (from_fp8_bytes(wq) * w_scale.float()[:, None]).reshape(Cout, KH, KW, Cin).permute(0, 3, 1, 2)
    xp = F.pad(xf.permute(0, 3, 1, 2), (pl, pr, pt, pb))
    y = F.conv2d(xp, wf, None, (sh, sw), 0, (dh, dw))[:, :, :Ho, :Wo].permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    y = _apply_act_ref(y, a)
    y = to_fp8_bytes(y / out_scale) if out_fp8 else y.to(odt)
    out[..., out_channel_offset:out_channel_offset + Cout] = y
    return out


def conv2d_nhwc_fp8_multi(x: torch.Tensor, x_scale: float, wq: torch.Tensor, kshape, w_scale: torch.Tensor,
                          bias: torch.Tensor, lo: torch.Tensor, segs, stride=(1, 1), pad=(0, 0, 0, 0), dilation=(1, 1),
                          chan_scale: torch.Tensor | None = None) -> None:
    """Horizontally fused sibling convs (``kernels/fp8.hip`` conv_lite_fp8, multi-output
    epilogue): one implicit GEMM over the concatenated filters ``wq`` [Cout_total, K]; output
    channels are clamped below by ``lo`` (0 = ReLU, -inf = none) and split into ``segs``:
    ``[(out, c0, c1, out_channel_offset, out_scale)]`` in channel order, ``out`` an NHWC
    buffer (e4m3 bytes with ``out_scale``, or bf16 when ``out_scale`` is None).  The tile is
    staged in bf16 and quantised per segment at the store."""
    N, H, W, Cin = x.shape
    Cout = wq.shape[0]
    KH, KW = kshape
    sh, sw = stride
    pt, pb, pl, pr = pad
    dh, dw = dilation
    Ho, Wo = conv_out_hw(H, W, KH, KW, sh, sw, pt, pl, dh, dw, pb, pr)
    for out, c0, c1, off, osc in segs:
        if tuple(out.shape[:3]) != (N, Ho, Wo) or off + (c1 - c0) > out.shape[3]:
            raise ValueError(f"conv2d_nhwc_fp8_multi: segment out {tuple(out.shape)} cannot hold [{c0}, {c1}) at {off}")
        if out.dtype != (torch.uint8 if osc is not None else (torch.bfloat16 if x.is_cuda else out.dtype)):
            raise ValueError("conv2d_nhwc_fp8_multi: segment dtype does not match its scale")
    if x.is_cuda:
        _check(x, "x", torch.uint8, x.device)
        _check(wq, "wq", torch.uint8, x.device)
        if wq.shape[1] != KH * KW * Cin:
            raise ValueError(f"conv2d_nhwc_fp8_multi: weight K {wq.shape[1]} != {KH}*{KW}*{Cin}")
        if chan_scale is None:
            chan_scale = (w_scale.float() * x_scale).contiguous()
        for t, nm in ((chan_scale, "chan_scale"), (bias, "bias"), (lo, "lo")):
            _check(t, nm, torch.float32, x.device)
        _hip().conv2d_nhwc_fp8_multi(
            x.data_ptr(), wq.data_ptr(), chan_scale.data_ptr(), bias.data_ptr(), lo.data_ptr(), N, H, W, Cin, Cout, KH,
            KW, sh, sw, pt, pl, dh, dw, Ho, Wo,
            [(o.data_ptr(), c0, c1, o.shape[-1], off, int(osc is None), 1.0 / osc if osc is not None else 1.0)
             for o, c0, c1, off, osc in segs], _stream(), 0)
        return
    y = conv2d_nhwc_fp8(x, x_scale, wq, kshape, w_scale, bias, stride, pad, dilation, None)  # fp32, no act
    y = torch.maximum(y, lo.float()).to(torch.bfloat16).float()  # the kernel stages the tile in bf16
    for out, c0, c1, off, osc in segs:
        v = y[..., c0:c1]
        out[..., off:off + c1 - c0] = to_fp8_bytes(v / osc) if osc is not None else v.to(out.dtype)


def gemm_fp8(x: torch.Tensor, x_scale: float, wq: torch.Tensor, w_scale: torch.Tensor, bias=None, act=None,
             out_scale: float | None = None, out: torch.Tensor | None = None, cfg: int = -1,
             chan_scale: torch.Tensor | None = None) -> torch.Tensor:
    """``act(x @ w^T * scales + bias)`` with fp8 operands; ``x`` [M, K] fp8 bytes or bf16."""
    x4 = x.reshape(x.shape[0], 1, 1, x.shape[1])
    o4 = None if out is None else out.reshape(out.shape[0], 1, 1, out.shape[1])
    y = conv2d_nhwc_fp8(x4, x_scale, wq, (1, 1), w_scale, bias, act=act, out_scale=out_scale, out=o4, cfg=cfg,
                        chan_scale=chan_scale)
    return y.reshape(x.shape[0], wq.shape[0])


def pool2d_nhwc_fp8(x: torch.Tensor, ksize, stride, pad=(0, 0, 0, 0), mode="max", rq: float = 1.0, out=None,
                    out_channel_offset: int = 0) -> torch.Tensor:
    """fp8 NHWC max/avg pool (avg excludes padding, TF semantics); output = pooled * rq."""
    N, H, W, C = x.shape
    kh, kw = ksize
    sh, sw = stride
    pt, pb, pl, pr = pad
    Ho = (H + pt + pb - kh) // sh + 1
    Wo = (W + pl + pr - kw) // sw + 1
    if out is None:
        out = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        out_channel_offset = 0
    if x.is_cuda:
        _check(x, "x", torch.uint8, x.device)
        _check(out, "out", torch.uint8, x.device)
        _hip().pool2d_nhwc_fp8(x.data_ptr(), out.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, pt, pl,
                               out.shape[-1], out_channel_offset, int(mode == "max"), float(rq), _stream())
        return out
    xf = from_fp8_bytes(x).permute(0, 3, 1, 2)
    if mode == "max":
        y = F.max_pool2d(F.pad(xf, (pl, pr, pt, pb), value=float("-inf")), (kh, kw), (sh, sw))
    else:
        s = F.avg_pool2d(F.pad(xf, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
        ones = F.pad(torch.ones_like(xf[:, :1]), (pl, pr, pt, pb))
        cnt = F.avg_pool2d(ones, (kh, kw), (sh, sw), divisor_override=1)
        y = s / cnt
    out[..., out_channel_offset:out_channel_offset + C] = to_fp8_bytes(y.permute(0, 2, 3, 1)[:, :Ho, :Wo] * rq)
    return out


def avgpool_bias_act(x: torch.Tensor, ksize, stride, pad, bias: torch.Tensor, act=None, out_scale: float | None = None,
                     out: torch.Tensor | None = None, out_channel_offset: int = 0) -> torch.Tensor:
    """``act(avgpool(x) + bias)`` over bf16 NHWC ``x`` (TF SAME average: divided by the
    in-bounds count), written as fp8 bytes of scale ``out_scale`` or as bf16 (None), into
    ``out`` at ``out_channel_offset`` (a concat buffer).  The second half of an
    AvgPool -> pointwise-conv branch computed as conv -> pool (``kernels/fp8.hip``
    ``avgpool_epi_kernel``)."""
    N, H, W, C = x.shape
    kh, kw = ksize
    sh, sw = stride
    pt, pb, pl, pr = pad
    Ho = (H + pt + pb - kh) // sh + 1
    Wo = (W + pl + pr - kw) // sw + 1
    a = act_code(act)
    out_fp8 = out_scale is not None
    if out is None:
        out = torch.empty((N, Ho, Wo, C), dtype=torch.uint8 if out_fp8 else (torch.bfloat16 if x.is_cuda else
                                                                               torch.float32), device=x.device)
        out_channel_offset = 0
    if tuple(out.shape[:3]) != (N, Ho, Wo) or out_channel_offset + C > out.shape[3]:
        raise ValueError(f"avgpool_bias_act: out {tuple(out.shape)} cannot hold [{N},{Ho},{Wo},{C}] at "
                         f"offset {out_channel_offset}")
    if x.is_cuda:
        _check(x, "x", torch.bfloat16, x.device)
        _check(bias, "bias", torch.float32, x.device)
        _check(out, "out", torch.uint8 if out_fp8 else torch.bfloat16, x.device)
        _hip().avgpool_bias_act(x.data_ptr(), bias.data_ptr(), out.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, pt,
                                pl, out.shape[-1], out_channel_offset, int(out_fp8),
                                1.0 / out_scale if out_fp8 else 1.0, a, _stream())
        return out
    xf = x.float().permute(0, 3, 1, 2)
    s = F.avg_pool2d(F.pad(xf, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
    cnt = F.avg_pool2d(F.pad(torch.ones_like(xf[:, :1]), (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
    y = _apply_act_ref((s / cnt).permute(0, 2, 3, 1)[:, :Ho, :Wo] + bias.float(), a)
    out[..., out_channel_offset:out_channel_offset + C] = to_fp8_bytes(y / out_scale) if out_fp8 else y.to(out.dtype)
    return out


def global_avgpool_fp8(x: torch.Tensor, scale: float, out=None) -> torch.Tensor:
    """[N, H, W, C] fp8 → [N, C] bf16 (device) / fp32 (host) mean * scale."""
    N, H, W, C = x.shape
    if x.is_cuda:
        _check(x, "x", torch.uint8, x.device)
        if out is None:
            out = torch.empty((N, C), dtype=torch.bfloat16, device=x.device)
        _hip().global_avgpool_fp8(x.data_ptr(), out.data_ptr(), N, H * W, C, float(scale), _stream())
        return out
    y = from_fp8_bytes(x).mean((1, 2)) * scale
    if out is not None:
        out.copy_(y)
        return out
    return y

