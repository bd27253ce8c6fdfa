"""Python entry points of the hand-written CDNA4 kernels.

Every op has exactly two implementations:

* **HBM tensors (``cuda``)** → the gfx950 HIP kernel in ``_hip`` (``kernels/*.hip``).  If
  the library is missing on a GPU machine the call raises — there is no silent PyTorch
  fallback on the device path.
* **host tensors** → a plain PyTorch fp32 reference with identical semantics, used by the
  CPU test-suite and as the numerics oracle for the GPU tests.

Shapes, dtypes, alignment and contiguity are validated on the host before any launch
(a malformed launch can fault the whole GPU).  All launches go to the caller's current
stream, so the ops are hipGraph-capturable.
"""
from __future__ import annotations

import copy
import functools
import os

import torch
import torch.nn.functional as F

from .. import _ext

ACT_NONE, ACT_RELU, ACT_GELU, ACT_SIGMOID, ACT_TANH, ACT_RELU6, ACT_DRELU = 0, 1, 2, 3, 4, 5, 6
_ACT_NAMES = {None: ACT_NONE, "none": ACT_NONE, "relu": ACT_RELU, "gelu": ACT_GELU, "gelu_tanh": ACT_GELU,
              "sigmoid": ACT_SIGMOID, "tanh": ACT_TANH, "relu6": ACT_RELU6, "drelu": ACT_DRELU}


def act_code(act) -> int:
    if isinstance(act, int):
        return act
    try:
        return _ACT_NAMES[act]
    except KeyError:
        raise ValueError(f"unknown activation {act!r}") from None


def _apply_act_ref(y: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return torch.relu(y)
    if act == ACT_GELU:
        return F.gelu(y, approximate="tanh")
    if act == ACT_SIGMOID:
        return torch.sigmoid(y)
    if act == ACT_TANH:
        return torch.tanh(y)
    if act == ACT_RELU6:
        return torch.clamp(y, 0, 6)
    return y


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


def _check(t: torch.Tensor, name: str, dtype=torch.bfloat16, device=None):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if device is not None and t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")


def _hip():
    return _ext.hip(required=True)


_ZERO_BIAS: dict = {}


def _zeros_bias(n: int, device) -> torch.Tensor:
    """Cached zero bias for bias-less layers (no allocation inside captured launches)."""
    key = (device, n)
    t = _ZERO_BIAS.get(key)
    if t is None:
        t = _ZERO_BIAS[key] = torch.zeros(n, dtype=torch.float32, device=device)
    return t


# ------------------------------------------------------------------------------ conv
# tile configs 0..4 are the register-staged igemm_bf16 tiles (-1: chosen by shape); the
# pipelined 256-pixel LDS-DMA kernel (igemm_v2) was in no default plan and was removed (r06)
def conv_out_hw(H, W, KH, KW, sh, sw, ph, pw, dh=1, dw=1, ph_hi=None, pw_hi=None):
    ph_hi = ph if ph_hi is None else ph_hi
    pw_hi = pw if pw_hi is None else pw_hi
    Ho = (H + ph + ph_hi - ((KH - 1) * dh + 1)) // sh + 1
    Wo = (W + pw + pw_hi - ((KW - 1) * dw + 1)) // sw + 1
    return Ho, Wo


def conv2d_nhwc(x: torch.Tensor, w_ohwi: torch.Tensor, bias: torch.Tensor | None = None,
                residual: torch.Tensor | None = None, stride=(1, 1), pad=(0, 0, 0, 0), dilation=(1, 1),
                act=None, out: torch.Tensor | None = None, out_channel_offset: int = 0, cfg: int = -1,
                out_scale: float | None = None) -> torch.Tensor:
    """NHWC conv, weights [Cout, KH, KW, Cin]; ``pad = (top, bottom, left, right)``.

    Fused epilogue ``act(conv + bias + residual)``.  With ``out`` given, the result is
    written at channel offset ``out_channel_offset`` of ``out`` (concat-by-stride-write).
    ``out_scale`` stores the result as OCP e4m3 bytes (``y / out_scale``, uint8): host
    reference only (the reference of ``conv2d_direct``'s fp8 epilogue).
    """
    a = act_code(act)
    N, H, W, Cin = x.shape
    Cout, KH, KW, Cin2 = w_ohwi.shape
    if Cin2 != Cin:
        raise ValueError(f"conv2d_nhwc: input has {Cin} channels, weights expect {Cin2}")
    sh, sw = stride
    pt, pb, pl, pr = pad
    dh, dw = dilation
    Ho, Wo = conv_out_hw(H, W, KH, KW, sh, sw, pt, pl, dh, dw, pb, pr)
    if out_scale is not None:
        if residual is not None:
            raise ValueError("conv2d_nhwc: fp8 output does not take a residual")
        if x.is_cuda:
            raise ValueError("conv2d_nhwc: e4m3 output is host-reference only on the implicit GEMM; "
                             "fp8 stems run on conv2d_direct")
    if out is None:
        odt = torch.uint8 if out_scale is not None else (x.dtype if x.is_cuda else torch.float32)
        out = torch.empty((N, Ho, Wo, Cout), dtype=odt, device=x.device)
        out_channel_offset = 0
    if out.shape[:3] != (N, Ho, Wo) or out_channel_offset + Cout > out.shape[3]:
        raise ValueError(f"conv2d_nhwc: out {tuple(out.shape)} cannot hold [{N},{Ho},{Wo},{Cout}] at "
                         f"offset {out_channel_offset}")
    if residual is not None and tuple(residual.shape) != (N, Ho, Wo, Cout):
        raise ValueError(f"conv2d_nhwc: residual {tuple(residual.shape)} != {(N, Ho, Wo, Cout)}")
    if x.is_cuda:
        for t, n in ((x, "x"), (w_ohwi, "w")):
            _check(t, n, device=x.device)
        _check(out, "out", torch.uint8 if out_scale is not None else torch.bfloat16, x.device)
        if residual is not None:
            _check(residual, "residual", device=x.device)
        if bias is not None:
            _check(bias, "bias", torch.float32, x.device)
            if bias.numel() != Cout:
                raise ValueError("conv2d_nhwc: bias size != Cout")
        else:
            bias = _zeros_bias(Cout, x.device)
        # bottom/right padding is implied by the kernel's bounds check (Ho/Wo carry it)
        _hip().conv2d_nhwc_bf16(x.data_ptr(), w_ohwi.data_ptr(), bias.data_ptr(), _ptr(residual), out.data_ptr(),
                                N, H, W, Cin, Cout, KH, KW, sh, sw, pt, pl, dh, dw, Ho, Wo, out.shape[3],
                                out_channel_offset, Cout if residual is None else residual.shape[3], a, _stream(), cfg)
        return out
    # host reference
    xn = x.float().permute(0, 3, 1, 2)
    xn = F.pad(xn, (pl, pr, pt, pb))
    y = F.conv2d(xn, w_ohwi.float().permute(0, 3, 1, 2), stride=(sh, sw), dilation=(dh, dw))
    y = y.permute(0, 2, 3, 1)
    if bias is not None:
        y = y + bias.float()
    if residual is not None:
        y = y + residual.float()
    y = _apply_act_ref(y, a)
    if out_scale is not None:
        from .fp8 import to_fp8_bytes

        out[..., out_channel_offset:out_channel_offset + Cout] = to_fp8_bytes(y / out_scale)
        return out
    out[..., out_channel_offset:out_channel_offset + Cout] = y.to(out.dtype)
    return out


def conv3x3_c64_eligible(x_shape, w_shape, stride, pad, dilation, residual, act) -> bool:
    """The persistent LDS-resident-weights kernel (kernels/conv3x3c64.hip): 3x3, stride 1,
    SAME padding, 64 -> 64 channels, no residual, bias (+ReLU) epilogue, H >= 8, W >= 32."""
    N, H, W, Cin = x_shape
    Cout, KH, KW, _ = w_shape
    return (Cin == 64 and Cout == 64 and (KH, KW) == (3, 3) and tuple(stride) == (1, 1) and tuple(pad) == (1, 1, 1, 1)
            and tuple(dilation) == (1, 1) and residual is None and act_code(act) in (ACT_NONE, ACT_RELU)
            and H >= 8 and W >= 32 and N * H * W * Cin * 2 < 2 ** 31)


_NUM_CU: dict = {}


class _PersistentCUs(dict):
    """CU count the persistent kernels size their grid to: the device's (caps of 224 / 192 /
    160 CUs, room for the sibling lane, measured -0.6 to -5 %: profiles/r04_ab)."""

    def __missing__(self, dev):
        self[dev] = torch.cuda.get_device_properties(dev).multi_processor_count
        return self[dev]


_NUM_CU = _PersistentCUs()


def conv3x3_c64(x: torch.Tensor, w_ohwi: torch.Tensor, bias: torch.Tensor, act=None, out: torch.Tensor | None = None,
                out_channel_offset: int = 0) -> torch.Tensor:
    """3x3 / s1 / SAME conv, 64 -> 64 channels, ``act(conv + bias)``; GPU: persistent
    kernel with the filter bank resident in LDS; host: the fp32 reference conv."""
    N, H, W, _ = x.shape
    a = act_code(act)
    if out is None:
        out = torch.empty((N, H, W, 64), dtype=x.dtype if x.is_cuda else torch.float32, device=x.device)
        out_channel_offset = 0
    if not conv3x3_c64_eligible(tuple(x.shape), tuple(w_ohwi.shape), (1, 1), (1, 1, 1, 1), (1, 1), None, a):
        raise ValueError(f"conv3x3_c64: unsupported shapes x {tuple(x.shape)} w {tuple(w_ohwi.shape)}")
    if out.shape[:3] != (N, H, W) or out_channel_offset + 64 > out.shape[3]:
        raise ValueError("conv3x3_c64: output buffer does not fit")
    if x.is_cuda:
        _check(x, "x", device=x.device)
        _check(w_ohwi, "w", device=x.device)
        _check(out, "out", device=x.device)
        _check(bias, "bias", torch.float32, x.device)
        dev = x.device.index if x.device.index is not None else torch.cuda.current_device()
        _hip().conv3x3c64_bf16(x.data_ptr(), w_ohwi.data_ptr(), bias.data_ptr(), out.data_ptr(), N, H, W, out.shape[3],
                               out_channel_offset, a, _NUM_CU[dev], _stream())
        return out
    return conv2d_nhwc(x, w_ohwi, bias, None, (1, 1), (1, 1, 1, 1), (1, 1), a, out=out,
                       out_channel_offset=out_channel_offset)


def bottleneck_tail(x2: torch.Tensor, res: torch.Tensor | None, w3: torch.Tensor, b3: torch.Tensor, w1: torch.Tensor,
                    b1: torch.Tensor, y3: torch.Tensor | None = None, y1: torch.Tensor | None = None,
                    xs: torch.Tensor | None = None, y3_decimated: bool = False):
    """Fused ResNet bottleneck block boundary (kernels/bottleneck.hip):
    ``y3 = relu(x2 @ w3^T + b3 + res)`` (1x1 expand CX -> 4 CX with residual) and
    ``y1 = relu(y3 @ w1^T + b1)`` (the next block's 1x1 reduce 4 CX -> CN); returns
    ``(y3, y1)``.  Variants: CX = 64 (stage 1) with CN = 64 or 128 (a stage-2 form with the
    weights streamed through LDS measured no faster than the two convs and was removed:
    profiles/r01_tail).  Dual form (stage 1's first block, stride-1
    projection shortcut): ``xs [..., 64]`` instead of ``res`` and ``w3 [256, 128]`` =
    [expand | projection] — ``y3 = relu([x2 | xs] @ w3^T + b3)`` (CN = 64).  Weights are 1x1
    OHWI squeezed ([out, in]), biases fp32.  GPU: one persistent kernel, y3 reused from LDS;
    host: the fp32 reference with y3 rounded to the output dtype before the second GEMM.

    ``y3_decimated``: ``x2`` is ``[N, H, W, 64]`` and only the even-(h, w) pixels of y3 are
    stored, compact as ``[N, H/2, W/2, 256]`` — for a y3 whose only other reader is a
    stride-2 1x1 projection shortcut (ResNet v1.5's stage-1 -> stage-2 boundary)."""
    lead = x2.shape[:-1]
    dec_hw = (0, 0)
    if y3_decimated:
        if x2.dim() != 4 or x2.shape[1] % 2 or x2.shape[2] % 2 or x2.shape[-1] != 64:
            raise ValueError("bottleneck_tail: decimated y3 needs x2 [N, H, W, 64] with even H, W")
        dec_hw = (x2.shape[1], x2.shape[2])
    dual = xs is not None
    cx = x2.shape[-1]
    co = 4 * cx
    cn = w1.shape[0]
    if (res is None) != dual:
        raise ValueError("bottleneck_tail: pass exactly one of res and xs")
    if (cx, dual, cn) not in ((64, True, 64), (64, False, 64), (64, False, 128)):
        raise ValueError(f"bottleneck_tail: unsupported variant x2 [..., {cx}], dual {dual}, reduce width {cn}")
    k3 = 2 * cx if dual else cx
    if (dual and tuple(xs.shape) != (*lead, cx)) or (not dual and tuple(res.shape) != (*lead, co)):
        raise ValueError(f"bottleneck_tail: the second input must be [..., {cx if dual else co}]")
    if tuple(w3.reshape(w3.shape[0], -1).shape) != (co, k3) or tuple(w1.reshape(cn, -1).shape) != (cn, co):
        raise ValueError(f"bottleneck_tail: weights must be [{co}, {k3}] and [{cn}, {co}], got {tuple(w3.shape)} "
                         f"{tuple(w1.shape)}")
    if b3.numel() != co or b1.numel() != cn:
        raise ValueError("bottleneck_tail: bias sizes must match the output channels")
    odt = x2.dtype if x2.is_cuda else torch.float32
    lead3 = (lead[0], dec_hw[0] // 2, dec_hw[1] // 2) if y3_decimated else lead
    y3 = torch.empty((*lead3, co), dtype=odt, device=x2.device) if y3 is None else y3
    y1 = torch.empty((*lead, cn), dtype=odt, device=x2.device) if y1 is None else y1
    if tuple(y3.shape) != (*lead3, co) or tuple(y1.shape) != (*lead, cn):
        raise ValueError("bottleneck_tail: output buffers do not fit")
    M = x2.numel() // cx
    second = xs if dual else res
    if x2.is_cuda:
        for t, n in ((x2, "x2"), (second, "xs" if dual else "res"), (w3, "w3"), (w1, "w1"), (y3, "y3"), (y1, "y1")):
            _check(t, n, device=x2.device)
        _check(b3, "b3", torch.float32, x2.device)
        _check(b1, "b1", torch.float32, x2.device)
        dev = x2.device.index if x2.device.index is not None else torch.cuda.current_device()
        _hip().bottleneck_tail_bf16(x2.data_ptr(), _ptr(xs), _ptr(res), w3.data_ptr(), b3.data_ptr(),
                                    w1.data_ptr(), b1.data_ptr(), y3.data_ptr(), y1.data_ptr(), M, cn,
                                    _NUM_CU[dev], _stream(), dec_hw[0], dec_hw[1])
        return y3, y1
    xin = torch.cat([x2.reshape(M, cx), xs.reshape(M, cx)], 1) if dual else x2.reshape(M, cx)
    a = xin.float() @ w3.reshape(co, k3).float().t() + b3.float()
    a = a.to(odt).float()  # the kernel rounds acc + bias first
    a = torch.relu(a if dual else a + res.reshape(M, co).float()).to(y3.dtype)
    y3.copy_(a.reshape(*lead, co)[:, ::2, ::2] if y3_decimated else a.reshape(y3.shape))
    b = torch.relu(a.float() @ w1.reshape(cn, co).float().t() + b1.float())
    y1.copy_(b.reshape(y1.shape).to(y1.dtype))
    return y3, y1


def bottleneck_chain(links, w1: torch.Tensor, b1: torch.Tensor, y1: torch.Tensor | None = None,
                     y3: torch.Tensor | None = None, y3_decimated: bool = False, store_y3: bool = True):
    """ResNet stage 1's residual stream recomputed instead of re-read (kernels/bottleneck_chain.hip):
    ``links`` = [(c1, x0, w_a, b_a), (c2, None, w_b, b_b), ...] (1 to 3), ``y = relu([c1|x0] .
    w_a^T + b_a)`` then ``y = relu(c_j . w_j^T + b_j + y)`` per further link — each link rounded
    exactly as ``bottleneck_tail`` rounds it (acc + b -> bf16, + residual, relu -> bf16) — then
    ``y1 = relu(y . w1^T + b1)``.  The last ``y`` is stored into ``y3`` only with
    ``store_y3`` (``y3_decimated``: the even-(h, w) pixels, compact).  Returns ``(y3 or None, y1)``.
    All sources [..., 64] of one pixel count; w_a [256, 128], the others [256, 64]; w1 [cn, 256]."""
    x0 = links[0][0]
    lead = x0.shape[:-1]
    M = x0.numel() // 64
    cn = w1.shape[0]
    if not 1 <= len(links) <= 3 or links[0][1] is None or any(l[1] is not None for l in links[1:]):
        raise ValueError("bottleneck_chain: 1 to 3 links, the first dual ([x | xs]), the others plain")
    for j, (x, xs, w, b) in enumerate(links):
        if x.shape[-1] != 64 or x.numel() != M * 64 or (xs is not None and tuple(xs.shape) != tuple(x.shape)):
            raise ValueError("bottleneck_chain: every source is [..., 64] over the same pixels")
        if tuple(w.reshape(w.shape[0], -1).shape) != (256, 128 if j == 0 else 64) or b.numel() != 256:
            raise ValueError(f"bottleneck_chain: link {j} weights must be [256, {128 if j == 0 else 64}]")
    if cn not in (64, 128) or tuple(w1.reshape(cn, -1).shape) != (cn, 256) or b1.numel() != cn:
        raise ValueError("bottleneck_chain: w1 must be [64 or 128, 256]")
    dec_hw = (0, 0)
    if y3_decimated:
        if x0.dim() != 4 or x0.shape[1] % 2 or x0.shape[2] % 2:
            raise ValueError("bottleneck_chain: decimated y3 needs [N, H, W, 64] sources with even H, W")
        dec_hw = (x0.shape[1], x0.shape[2])
    odt = x0.dtype if x0.is_cuda else torch.float32
    lead3 = (lead[0], dec_hw[0] // 2, dec_hw[1] // 2) if y3_decimated else lead
    if store_y3 and y3 is None:
        y3 = torch.empty((*lead3, 256), dtype=odt, device=x0.device)
    y1 = torch.empty((*lead, cn), dtype=odt, device=x0.device) if y1 is None else y1
    if (store_y3 and tuple(y3.shape) != (*lead3, 256)) or tuple(y1.shape) != (*lead, cn):
        raise ValueError("bottleneck_chain: output buffers do not fit")
    if x0.is_cuda:
        for j, (x, xs, w, b) in enumerate(links):
            for t, n in ((x, "x"), (w, "w")) + (((xs, "xs"),) if xs is not None else ()):
                _check(t, f"link {j} {n}", device=x0.device)
            _check(b, f"link {j} bias", torch.float32, x0.device)
        _check(w1, "w1", device=x0.device)
        _check(b1, "b1", torch.float32, x0.device)
        _check(y1, "y1", device=x0.device)
        if store_y3:
            _check(y3, "y3", device=x0.device)
        dev = x0.device.index if x0.device.index is not None else torch.cuda.current_device()
        _hip().bottleneck_chain_bf16([(x.data_ptr(), _ptr(xs), w.data_ptr(), b.data_ptr()) for x, xs, w, b in links],
                                     w1.data_ptr(), b1.data_ptr(), y3.data_ptr() if store_y3 else 0, y1.data_ptr(), M,
                                     cn, _NUM_CU[dev], _stream(), dec_hw[0], dec_hw[1])
        return (y3 if store_y3 else None), y1
    y = None
    rdt = y1.dtype  # each link's y3 rounded as the unfused tail's y3 buffer would hold it
    for x, xs, w, b in links:
        xin = torch.cat([x.reshape(M, 64), xs.reshape(M, 64)], 1) if xs is not None else x.reshape(M, 64)
        a = (xin.float() @ w.reshape(256, -1).float().t() + b.float()).to(odt).float()
        y = torch.relu(a if y is None else a + y).to(rdt).float()
    if store_y3:
        y3.copy_(y.reshape(*lead, 256)[:, ::2, ::2] if y3_decimated else y.reshape(y3.shape))
    y1.copy_(torch.relu(y @ w1.reshape(cn, 256).float().t() + b1.float()).reshape(y1.shape).to(y1.dtype))
    return (y3 if store_y3 else None), y1


def gemm(x: torch.Tensor, w_nk: torch.Tensor, bias: torch.Tensor | None = None, residual: torch.Tensor | None = None,
         act=None, out: torch.Tensor | None = None, cfg: int = -1) -> torch.Tensor:
    """``act(x[M,K] @ w[N,K]^T + bias + residual)``; leading dims of x are flattened."""
    a = act_code(act)
    lead = x.shape[:-1]
    K = x.shape[-1]
    N, K2 = w_nk.shape
    if K != K2:
        raise ValueError(f"gemm: K mismatch {K} vs {K2}")
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if out is None:
        out = torch.empty((*lead, N), dtype=x.dtype if x.is_cuda else torch.float32, device=x.device)
    out2 = out.reshape(M, N)
    if residual is not None and residual.numel() != M * N:
        raise ValueError("gemm: residual shape mismatch")
    if x.is_cuda:
        _check(x2, "x", device=x.device)
        _check(w_nk, "w", device=x.device)
        _check(out2, "out", device=x.device)
        if bias is not None:
            _check(bias, "bias", torch.float32, x.device)
        else:
            bias = _zeros_bias(N, x.device)
        if residual is not None:
            _check(residual, "residual", device=x.device)
        _hip().gemm_bf16(x2.data_ptr(), w_nk.data_ptr(), bias.data_ptr(), _ptr(residual), out2.data_ptr(), M, N, K, K,
                         N, N, a, _stream(), cfg)
        return out
    y = x2.float() @ w_nk.float().t()
    if bias is not None:
        y = y + bias.float()
    if residual is not None:
        y = y + residual.reshape(M, N).float()
    out2.copy_(_apply_act_ref(y, a).to(out.dtype))
    return out


# ------------------------------------------------------------------------------ gemm_train
_TR_KTILE_US = 0.45       # one 128x128x64 K step, two workgroups sharing a CU (2-stage ring)
_TR_KTILE_DEEP_US = 0.3   # the same with the CU to itself (4-stage ring, grids <= one per CU)
_TR_SLOTS = 512           # resident 128x128 workgroups (2 per CU)


def _tr_time(tiles: int, per: int, se: int, num_cu: int = 256) -> float:
    wgs = tiles * se
    if wgs <= num_cu:
        return per * _TR_KTILE_DEEP_US
    return -(-wgs // _TR_SLOTS) * per * _TR_KTILE_US


def gemm_train_splits(M: int, N: int, K: int) -> int:
    """Split-K factor for ``gemm_train``: rounds of resident 128x128 workgroups times K
    steps, plus the fp32 slab round trip of the reduction and its launch."""
    tiles = -(-M // 128) * -(-N // 128)
    nk = -(-K // 64)
    best_s, best_t = 1, _tr_time(tiles, nk, 1)
    for s in (2, 3, 4, 6, 8, 12, 16, 24, 32):
        if s > nk:
            break
        per = -(-nk // s)
        se = -(-nk // per)
        t = _tr_time(tiles, per, se) + se * M * N * 8 / _PP_SPLIT_BW + 2.0
        if t < 0.9 * best_t:
            best_s, best_t = se, t
    return best_s


def gemm_train(x: torch.Tensor, w: torch.Tensor, *, x_t: bool = False, w_t: bool = False,
               bias: torch.Tensor | None = None, mask: torch.Tensor | None = None, act=None,
               out: torch.Tensor | None = None, out_dtype=torch.bfloat16, splits: int | None = None,
               ws: torch.Tensor | None = None, colsum: torch.Tensor | None = None) -> torch.Tensor:
    """``epi(X @ W^T)`` on the layout-general training GEMM (``kernels/gemm_train.hip``).

    ``X`` is ``x`` [M, K] (K-contiguous) or, with ``x_t``, ``x`` stored [K, M]; ``W`` is
    ``w`` [N, K] or, with ``w_t``, ``w`` stored [K, N] — so a dense layer's three GEMMs need
    no transposed copies: forward ``gemm_train(h, W)``, dX ``gemm_train(dA, W, w_t=True)``,
    dW ``gemm_train(dA, h, x_t=True, w_t=True, out_dtype=torch.float32)``.  ``mask`` (bf16
    [M, N], e.g. the layer input) applies the ReLU backward ``mask > 0 ? y : 0``; ``out`` may
    be a row-strided view.  fp32 output takes no activation.  ``splits`` > 1 runs split-K
    (None: cost model) with an fp32 workspace ``ws`` (>= splits*M*N floats).  ``colsum``
    (fp32 [ceil(M/128), N], bf16 output, no split) receives every 128-row tile's column sums
    of the stored values — ``colsum_reduce`` turns them into the next layer's bias gradient.
    K must be a multiple of 8 (a partial last K tile reads zeros)."""
    a = act_code(act)
    if mask is not None:
        a = ACT_DRELU
    M, K = (x.shape[1], x.shape[0]) if x_t else (x.shape[0], x.shape[1])
    N, K2 = (w.shape[1], w.shape[0]) if w_t else (w.shape[0], w.shape[1])
    if K != K2:
        raise ValueError(f"gemm_train: K mismatch {K} vs {K2}")
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=x.device)
    if tuple(out.shape) != (M, N):
        raise ValueError(f"gemm_train: out shape {tuple(out.shape)} != {(M, N)}")
    f32 = out.dtype == torch.float32
    if not x.is_cuda:  # reference path (CPU): same math in fp32
        X = x.float().t() if x_t else x.float()
        W = w.float() if w_t else w.float().t()
        y = X @ W
        if bias is not None:
            y = y + bias.float()
        if mask is not None:
            y = torch.where(mask.float() > 0, y, torch.zeros_like(y))
        else:
            y = _apply_act_ref(y, a)
        out.copy_(y.to(out.dtype))
        if colsum is not None:
            yq = out.float()
            for t in range(colsum.shape[0]):
                colsum[t].copy_(yq[t * 128:(t + 1) * 128].sum(0))
        return out
    for t, nm in ((x, "x"), (w, "w")):  # row-strided views are fine (ld = stride(0))
        if t.dtype != torch.bfloat16 or t.device != x.device or t.dim() != 2 or t.stride(1) != 1:
            raise ValueError(f"gemm_train: {nm} must be a bf16 [rows, cols] view with contiguous rows on {x.device}")
    if out.stride(1) != 1:
        raise ValueError("gemm_train: out rows must be contiguous")
    if bias is not None:
        _check(bias, "bias", torch.float32, x.device)
    if mask is not None:
        _check(mask, "mask", device=x.device)
        if tuple(mask.shape) != (M, N) or mask.stride(1) != 1:
            raise ValueError("gemm_train: mask must be [M, N] with contiguous rows")
    if colsum is not None:
        if f32 or tuple(colsum.shape) != (-(-M // 128), N) or colsum.dtype != torch.float32 or not colsum.is_contiguous():
            raise ValueError("gemm_train: colsum must be contiguous fp32 [ceil(M/128), N] with bf16 output")
        splits = 1
    s = gemm_train_splits(M, N, K) if splits is None else int(splits)
    s = _hip().gemm_train_splits(K, s)
    wsp = 0
    if s > 1:
        need = s * M * N
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.float32, device=x.device)
        wsp = ws.data_ptr()
    _hip().gemm_train(x.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(mask), out.data_ptr(), M, N, K, x.stride(0),
                      w.stride(0), out.stride(0), mask.stride(0) if mask is not None else 0, bool(x_t), bool(w_t), a,
                      f32, s, wsp, _ptr(colsum), _stream())
    return out


def colsum_reduce(part: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """``out[n] = sum_t part[t, n]`` in fixed order (``gemm_train``'s per-tile column sums ->
    a bias gradient); ``part`` may be a column slice of a wider partial buffer."""
    T, N = part.shape
    if out.numel() != N:
        raise ValueError("colsum_reduce: out must hold N floats")
    if not part.is_cuda:
        out.copy_(part.sum(0).reshape(out.shape))
        return out
    if part.stride(1) != 1 or not out.is_contiguous():
        raise ValueError("colsum_reduce: contiguous rows / output")
    _hip().colsum_reduce(part.data_ptr(), T, part.stride(0), N, out.data_ptr(), _stream())
    return out


# ------------------------------------------------------------------------------ gemm_pp
_PP_KTILE_US = 1.5    # one 256x256x64 K step of one workgroup (measured: 1.39 PF at 8192^3)
_PP_SPLIT_BW = 5.0e6  # bytes per microsecond of the fp32 partial round trip (write + read)


def gemm_pp_splits(M: int, N: int, K: int, num_cu: int = 256) -> int:
    """Split-K factor for ``gemm_pp`` from a small cost model: waves of 256x256 tiles times
    K steps, plus the fp32 partial slices written and re-read by the reduction and one
    extra launch.  Splits only when that wins by >10 % (small-M heads, few-tile shapes)."""
    tiles = -(-M // 256) * -(-N // 256)
    nk = K // 64
    best_s, best_t = 1, -(-tiles // num_cu) * nk * _PP_KTILE_US
    for s in range(2, min(16, nk) + 1):
        per = -(-nk // s)
        se = -(-nk // per)
        t = -(-tiles * se // num_cu) * per * _PP_KTILE_US + 2.0 * se * M * N * 4 / _PP_SPLIT_BW + 2.0
        if t < 0.9 * best_t:
            best_s, best_t = se, t
    return best_s


def gemm_pp(x: torch.Tensor, w_nk: torch.Tensor, bias: torch.Tensor | None = None,
            residual: torch.Tensor | None = None, act=None, out: torch.Tensor | None = None,
            splits: int | None = None, out_col: int = 0, ws: torch.Tensor | None = None) -> torch.Tensor:
    """``act(x[M,K] @ w[N,K]^T + bias (+ residual))`` on the ping-pong 256x256 MFMA kernel
    (``kernels/gemm_pp.hip``).  ``out`` may be wider than N (``out_col`` = first column:
    concat-by-stride-write).  ``splits`` > 1 runs split-K (None: cost model) through the
    fp32 workspace ``ws`` (>= splits*M*N floats); without one a temporary is allocated per
    call — stream-ordered, and inside hipGraph capture it comes from the graph's pool."""
    a = act_code(act)
    lead = x.shape[:-1]
    K = x.shape[-1]
    N, K2 = w_nk.shape
    if K != K2:
        raise ValueError(f"gemm_pp: K mismatch {K} vs {K2}")
    x2 = x.reshape(-1, K)
    M = x2.shape[0]
    if out is None:
        out = torch.empty((*lead, N), dtype=x.dtype if x.is_cuda else torch.float32, device=x.device)
    ldy = out.shape[-1]
    out2 = out.reshape(-1, ldy)
    if out2.shape[0] != M or out_col + N > ldy:
        raise ValueError("gemm_pp: output shape mismatch")
    if residual is not None and residual.numel() != M * N:
        raise ValueError("gemm_pp: residual shape mismatch")
    if x.is_cuda:
        if K % 64 or N % 8 or ldy % 8 or out_col % 8:
            raise ValueError("gemm_pp: needs K % 64 == 0 and N, ldy, out_col % 8 == 0")
        _check(x2, "x", device=x.device)
        _check(w_nk, "w", device=x.device)
        _check(out2, "out", device=x.device)
        if bias is not None:
            _check(bias, "bias", torch.float32, x.device)
        if residual is not None:
            _check(residual, "residual", device=x.device)
        if splits is None:
            splits = gemm_pp_splits(M, N, K)
        splits = _hip().gemm_pp_splits(K, splits)
        if splits > 1:
            if ws is None:
                ws = torch.empty(splits * M * N, dtype=torch.float32, device=x.device)
            elif ws.dtype != torch.float32 or ws.device != x.device or ws.numel() < splits * M * N:
                raise ValueError(f"gemm_pp: workspace needs {splits * M * N} fp32 elements on {x.device}")
        else:
            ws = None
        _hip().gemm_pp(x2.data_ptr(), w_nk.data_ptr(), _ptr(bias), _ptr(residual), out2.data_ptr(), M, N, K, K, K,
                       ldy, out_col, N, a, splits, _ptr(ws), _stream())
        return out
    y = x2.float() @ w_nk.float().t()
    if bias is not None:
        y = y + bias.float()
    if a == ACT_DRELU:  # the residual operand is the ReLU mask source, not an addend
        if residual is None:
            raise ValueError("gemm_pp: act 'drelu' needs the mask operand (residual)")
        out2[:, out_col:out_col + N] = torch.where(residual.reshape(M, N).float() > 0, y, 0.0).to(out.dtype)
        return out
    if residual is not None:
        y = y + residual.reshape(M, N).float()
    out2[:, out_col:out_col + N] = _apply_act_ref(y, a).to(out.dtype)
    return out


def conv_pp_ktab(srcs) -> torch.Tensor:
    """Host-built K-tile table of ``conv_pp``: for every 64-wide K tile (source, kh, kw,
    channel chunk order) the byte delta of its input rows relative to the receptive-field
    origin, and ``src << 20 | kh*dh << 10 | kw*dw``.  ``srcs``: (H, W, C, KH, KW, dh, dw)."""
    rows = []
    for si, (H, W, C, KH, KW, dh, dw) in enumerate(srcs):
        for kh in range(KH):
            for kw in range(KW):
                for cc in range(C // 64):
                    rows.append((((kh * dh * W + kw * dw) * C + cc * 64) * 2, (si << 20) | (kh * dh << 10) | (kw * dw)))
    return torch.tensor(rows, dtype=torch.int32)


class ConvPP:
    """A planned ``conv_lite`` launch (kernels/conv_pp.hip): implicit-GEMM NHWC convolution
    of one or two sources into one accumulator on the 4-wave 128x128 LDS-DMA tile (``tile``
    2; 4..6 are diagnostic variants).  The ping-pong / wide / wave-split / two-wave /
    deeper-prefetch tiles measured slower and were removed (``kernels/conv_pp.hip``).

    ``srcs``: [(x_shape NHWC, (KH, KW), (sh, sw), (pt, pl), (dh, dw))]; the weight is the
    concatenation of the sources' OHWI filters, [Cout, sum KH*KW*C] bf16; a second source
    must be 1x1, unpadded and in range (a projection shortcut).  The K-tile table is built
    once (a device tensor kept on the object)."""

    def __init__(self, srcs, Cout: int, out_hw, device, tile: int | None = None, splits: int | None = None):
        self.srcs = [(tuple(xs), tuple(k), tuple(st), tuple(pd), tuple(dl)) for xs, k, st, pd, dl in srcs]
        self.N = self.srcs[0][0][0]
        self.OH, self.OW = out_hw
        self.Cout = Cout
        self.K = sum(k[0] * k[1] * xs[3] for xs, k, _, _, _ in self.srcs)
        for xs, _, _, _, _ in self.srcs:
            if xs[3] % 64 or xs[0] != self.N:
                raise ValueError("conv_pp: channels must be multiples of 64 and batches equal")
        if Cout % 8:
            raise ValueError("conv_pp: Cout % 8")
        self.M = self.N * self.OH * self.OW
        self.tile = 2 if tile is None else tile
        # (4..6: diagnostic variants for bench/conv_layer_probe.py, outputs meaningless)
        if self.tile not in (2, 4, 5, 6) or (splits or 1) != 1 or (self.tile != 2 and len(self.srcs) != 1):
            raise ValueError("conv_pp: only the conv_lite tile (2) without split-K remains")
        if len(self.srcs) == 2:
            (xs1, k1, st1, pd1, dl1) = self.srcs[1]
            if tuple(k1) != (1, 1) or tuple(pd1) != (0, 0) or (self.OH - 1) * st1[0] >= xs1[1] \
                    or (self.OW - 1) * st1[1] >= xs1[2]:
                raise ValueError("conv_pp: the 4-wave tile's second source must be 1x1, unpadded, in range")
        self.splits = 1
        self.ktab = conv_pp_ktab([(xs[1], xs[2], xs[3], k[0], k[1], dl[0], dl[1])
                                  for xs, k, _, _, dl in self.srcs]).to(device)
        self.ws = (torch.empty(self.splits * self.M * Cout, dtype=torch.float32, device=device)
                   if self.splits > 1 else None)

    def for_batch(self, n: int) -> "ConvPP":
        """The same convolution planned for ``n`` images (a batch slice: the compiler's
        batch-slice chain); shares the K-tile table and the split-K workspace."""
        if n == self.N:
            return self
        subs = self.__dict__.setdefault("_subs", {})
        sub = subs.get(n)
        if sub is None:
            sub = copy.copy(self)
            sub.srcs = [((n, *xs[1:]), k, st, pd, dl) for xs, k, st, pd, dl in self.srcs]
            sub.N, sub.M, sub._subs = n, n * self.OH * self.OW, {}
            if n > self.N:
                raise ValueError("conv_pp: a batch slice larger than the planned batch")
            subs[n] = sub
        return sub

    def __call__(self, xs, w, bias=None, residual=None, act=None, out=None, out_channel_offset: int = 0):
        if len(xs) != len(self.srcs):
            raise ValueError("conv_pp: source count")
        if xs and xs[0].dim() == 4 and xs[0].shape[0] != self.N:
            return self.for_batch(int(xs[0].shape[0]))(xs, w, bias, residual, act, out, out_channel_offset)
        for x, (shape, *_r) in zip(xs, self.srcs):
            if tuple(x.shape) != shape:
                raise ValueError(f"conv_pp: input shape {tuple(x.shape)} != planned {shape}")
        if out is None:
            out = torch.empty((self.N, self.OH, self.OW, self.Cout), dtype=torch.bfloat16, device=xs[0].device)
        ldy = out.shape[-1]
        if tuple(out.shape[:3]) != (self.N, self.OH, self.OW) or out_channel_offset + self.Cout > ldy:
            raise ValueError("conv_pp: output shape mismatch")
        if tuple(w.shape) != (self.Cout, self.K):
            raise ValueError(f"conv_pp: weight {tuple(w.shape)} != ({self.Cout}, {self.K})")
        if not xs[0].is_cuda:
            return self._reference(xs, w, bias, residual, act, out, out_channel_offset)
        for i, x in enumerate(xs):
            _check(x, f"x{i}", device=out.device)
        _check(w, "w", device=out.device)
        _check(out, "out", device=out.device)
        if bias is not None:
            _check(bias, "bias", torch.float32, out.device)
        if residual is not None:
            _check(residual, "residual", device=out.device)
            if residual.numel() != self.M * self.Cout:
                raise ValueError("conv_pp: residual shape")
        srcs = [(x.data_ptr(), self.N, sh[1], sh[2], sh[3], k[0], k[1], st[0], st[1], pd[0], pd[1], dl[0], dl[1])
                for x, (sh, k, st, pd, dl) in zip(xs, self.srcs)]
        _hip().conv_pp(srcs, self.ktab.data_ptr(), w.data_ptr(), _ptr(bias), _ptr(residual), out.data_ptr(),
                       self.N, self.OH, self.OW, self.Cout, ldy, out_channel_offset, self.Cout, act_code(act),
                       self.tile, self.splits, _ptr(self.ws), _stream())
        return out

    def _reference(self, xs, w, bias, residual, act, out, coff):
        """fp32 host reference (CPU tests): the sum of the sources' convolutions."""
        import torch.nn.functional as F

        y = 0
        k0 = 0
        for x, (sh, (KH, KW), (s_h, s_w), (pt, pl), (dh, dw)) in zip(xs, self.srcs):
            C = sh[3]
            wk = w[:, k0:k0 + KH * KW * C].float().reshape(self.Cout, KH, KW, C).permute(0, 3, 1, 2)
            k0 += KH * KW * C
            xi = x.float().permute(0, 3, 1, 2)
            ph_hi = max(0, (self.OH - 1) * s_h + (KH - 1) * dh + 1 - sh[1] - pt)
            pw_hi = max(0, (self.OW - 1) * s_w + (KW - 1) * dw + 1 - sh[2] - pl)
            xi = F.pad(xi, (pl, pw_hi, pt, ph_hi))
            yi = F.conv2d(xi, wk, stride=(s_h, s_w), dilation=(dh, dw))[:, :, :self.OH, :self.OW]
            y = y + yi
        y = y.permute(0, 2, 3, 1)
        if bias is not None:
            y = y + bias.float()
        if residual is not None:
            y = y + residual.reshape(y.shape).float()
        out[..., coff:coff + self.Cout] = _apply_act_ref(y, act_code(act)).to(out.dtype)
        return out


# ------------------------------------------------------------------------------ preprocess
def preprocess_images(images_u8: torch.Tensor, out_hw=(224, 224), mean=(117.0, 117.0, 117.0),
                      std=(1.0, 1.0, 1.0), align_corners=False, half_pixel_centers=False,
                      out: torch.Tensor | None = None, s2d: bool = False) -> torch.Tensor:
    """uint8 [B,H,W,3] → resize (TF ResizeBilinear) → (v-mean)/std → bf16.

    Layout ``[B,Ho,Wo,8]`` (channels 3..7 zero), or with ``s2d`` the 2x2 space-to-depth
    layout ``[B,ceil(Ho/2),ceil(Wo/2),16]`` consumed by the stride-2 stem conv
    (``s2d_stem_weights``); an odd size zero-fills the pixels past the image."""
    if images_u8.dtype != torch.uint8 or images_u8.dim() != 4 or images_u8.shape[3] != 3:
        raise ValueError("preprocess_images expects uint8 [B,H,W,3]")
    B, Hi, Wi, _ = images_u8.shape
    Ho, Wo = out_hw
    oshape = (B, (Ho + 1) // 2, (Wo + 1) // 2, 16) if s2d else (B, Ho, Wo, 8)
    if out is None:
        out = torch.empty(oshape, dtype=torch.bfloat16 if images_u8.is_cuda else torch.float32,
                          device=images_u8.device)
    if tuple(out.shape) != oshape:
        raise ValueError(f"preprocess_images: out must be {oshape}, got {tuple(out.shape)}")
    if images_u8.is_cuda:
        if not images_u8.is_contiguous():
            raise ValueError("preprocess_images: input must be contiguous")
        _check(out, "out", device=images_u8.device)
        _hip().preprocess_u8_to_bf16(images_u8.data_ptr(), out.data_ptr(), B, Hi, Wi, Ho, Wo, int(align_corners),
                                     int(half_pixel_centers), float(mean[0]), float(mean[1]), float(mean[2]),
                                     1.0 / std[0], 1.0 / std[1], 1.0 / std[2], Hi * Wi * 3, int(s2d), _stream())
        return out
    from ..graph.ops_nn import resize_bilinear_tf

    y = resize_bilinear_tf(images_u8.float(), Ho, Wo, align_corners, half_pixel_centers)
    y = (y - torch.tensor(mean)) / torch.tensor(std)
    out.zero_()
    if s2d:
        Hb, Wb = (Ho + 1) // 2, (Wo + 1) // 2
        y = F.pad(y, (0, 0, 0, 2 * Wb - Wo, 0, 2 * Hb - Ho))
        blk = y.reshape(B, Hb, 2, Wb, 2, 3).permute(0, 1, 3, 2, 4, 5).reshape(B, Hb, Wb, 12)
        out[..., :12] = blk.to(out.dtype)
    else:
        out[..., :3] = y.to(out.dtype)
    return out


def s2d_stem_weights(w_hwio: torch.Tensor, H: int, W: int, pads):
    """Rewrites a stride-2 KxK conv over RGB (pads top/left even) as a stride-1
    ceil(K/2)² conv over the 2x2 space-to-depth input (16 channels, 12 used).

    Returns ``(w_ohwi [Cout, KBH, KBW, 16], block_pads (t, b, l, r))``.  Cuts the stem's
    MFMA work from K = 7·7·8 = 392 to 4·4·16 = 256 and makes every 16-B im2col load useful.
    """
    KH, KW, C, Cout = w_hwio.shape
    pt, pb, pl, pr = pads
    if C != 3 or pt % 2 or pl % 2:
        raise ValueError("s2d stem needs RGB input and even top/left padding")
    KBH, KBW = (KH + 1) // 2, (KW + 1) // 2
    w2 = torch.zeros(Cout, KBH, KBW, 16, dtype=torch.float32)
    wf = w_hwio.float()
    for kh in range(KH):
        for kw in range(KW):
            ch = ((kh % 2) * 2 + (kw % 2)) * 3
            w2[:, kh // 2, kw // 2, ch:ch + 3] = wf[kh, kw].t()
    Ho = (H + pt + pb - KH) // 2 + 1
    Wo = (W + pl + pr - KW) // 2 + 1
    Hb, Wb = (H + 1) // 2, (W + 1) // 2  # an odd size's last block is zero-filled past the image
    pt_b, pl_b = pt // 2, pl // 2
    pb_b = Ho - 1 + KBH - Hb - pt_b
    pr_b = Wo - 1 + KBW - Wb - pl_b
    if pb_b < 0 or pr_b < 0:
        raise ValueError("s2d stem: negative block padding")
    return w2, (pt_b, pb_b, pl_b, pr_b)


# ------------------------------------------------------------------------------ pooling
def pool2d_nhwc(x: torch.Tensor, ksize, stride, pad=(0, 0, 0, 0), mode="max", out=None, out_channel_offset=0):
    N, H, W, C = x.shape
    kh, kw = ksize
    sh, sw = stride
    pt, pb, pl, pr = pad
    Ho = (H + pt + pb - kh) // sh + 1
    Wo = (W + pl + pr - kw) // sw + 1
    if out is None:
        out = torch.empty((N, Ho, Wo, C), dtype=x.dtype, device=x.device)
        out_channel_offset = 0
    if x.is_cuda:
        _check(x, "x", device=x.device)
        _check(out, "out", device=x.device)
        _hip().pool2d_nhwc_bf16(x.data_ptr(), out.data_ptr(), N, H, W, C, Ho, Wo, kh, kw, sh, sw, pt, pl,
                                int(mode == "max"), out.shape[3], out_channel_offset, _stream())
        return out
    xn = x.float().permute(0, 3, 1, 2)
    if mode == "max":
        y = F.max_pool2d(F.pad(xn, (pl, pr, pt, pb), value=float("-inf")), (kh, kw), (sh, sw))
    else:
        s = F.avg_pool2d(F.pad(xn, (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
        c = F.avg_pool2d(F.pad(torch.ones_like(xn[:, :1]), (pl, pr, pt, pb)), (kh, kw), (sh, sw), divisor_override=1)
        y = s / c
    out[..., out_channel_offset:out_channel_offset + C] = y.permute(0, 2, 3, 1).to(out.dtype)
    return out


def global_avgpool(x: torch.Tensor, out=None) -> torch.Tensor:
    N, H, W, C = x.shape
    if out is None:
        out = torch.empty((N, C), dtype=x.dtype, device=x.device)
    if x.is_cuda:
        _check(x, "x", device=x.device)
        _check(out, "out", device=x.device)
        _hip().global_avgpool_bf16(x.data_ptr(), out.data_ptr(), N, H * W, C, _stream())
        return out
    out.copy_(x.float().mean((1, 2)).to(out.dtype))
    return out


# ------------------------------------------------------------------------------ softmax/top-k
def softmax_topk(logits: torch.Tensor, k: int, want_probs: bool = False, vals=None, idxs=None, probs=None):
    """Row softmax + top-k → (values fp32 [R,k], indices int32 [R,k], probs or None)."""
    R, C = logits.shape
    dev = logits.device
    if vals is None:
        vals = torch.empty((R, k), dtype=torch.float32, device=dev)
    if idxs is None:
        idxs = torch.empty((R, k), dtype=torch.int32, device=dev)
    if want_probs and probs is None:
        probs = torch.empty((R, C), dtype=logits.dtype, device=dev)
    if logits.is_cuda:
        if logits.stride(1) != 1:
            raise ValueError("softmax_topk: logits rows must be contiguous")
        _check(vals, "vals", torch.float32, dev)
        _check(idxs, "idxs", torch.int32, dev)
        _hip().softmax_topk_bf16(logits.data_ptr(), R, C, logits.stride(0), k, vals.data_ptr(), idxs.data_ptr(),
                                 _ptr(probs), _stream())
        return vals, idxs, probs
    p = torch.softmax(logits.float(), -1)
    v, i = torch.topk(p, k, -1)
    vals.copy_(v)
    idxs.copy_(i.to(torch.int32))
    if probs is not None:
        probs.copy_(p.to(probs.dtype))
    return vals, idxs, probs


# ------------------------------------------------------------------------------ attention
def attention(qkv: torch.Tensor, ids: torch.Tensor | None, batch: int, seq: int, heads: int, pad_id: int = 0,
              scale: float | None = None, out: torch.Tensor | None = None,
              cu_seqlens: torch.Tensor | None = None) -> torch.Tensor:
    """Multi-head self-attention over the fused QKV projection output.

    Padded batch: ``qkv`` [B*S, 3*H*64] bf16 (Q|K|V blocks, head h at h*64), ``ids`` [B*S]
    int32 token ids (keys whose id == ``pad_id`` are masked).  Packed batch
    (``cu_seqlens`` [B+1] int32 given, ``seq`` = the longest sequence): sequence b is rows
    ``cu[b]:cu[b+1]`` of ``qkv``, no padding; rows past ``cu[B]`` are left untouched.
    Returns ctx [rows, H*64]."""
    T = qkv.shape[0] if cu_seqlens is not None else batch * seq
    Dh = qkv.shape[1] // (3 * heads)
    if qkv.shape != (T, 3 * heads * Dh):
        raise ValueError(f"attention: qkv shape {tuple(qkv.shape)} != {(T, 3 * heads * Dh)}")
    if cu_seqlens is None and (ids is None or ids.numel() != T):
        raise ValueError("attention: ids must have B*S entries")
    if cu_seqlens is not None and cu_seqlens.numel() != batch + 1:
        raise ValueError("attention: cu_seqlens must have B+1 entries")
    scale = (1.0 / Dh ** 0.5) if scale is None else scale
    if out is None:
        out = torch.empty((T, heads * Dh), dtype=qkv.dtype, device=qkv.device)
    if qkv.is_cuda:
        _check(qkv, "qkv", device=qkv.device)
        _check(out, "out", device=qkv.device)
        if cu_seqlens is not None:
            _check(cu_seqlens, "cu_seqlens", torch.int32, qkv.device)
        else:
            _check(ids, "ids", torch.int32, qkv.device)
        _hip().attention_fwd_bf16(qkv.data_ptr(), _ptr(ids) if cu_seqlens is None else 0, _ptr(cu_seqlens),
                                  out.data_ptr(), batch, seq, heads, Dh, pad_id, float(scale), _stream())
        return out
    if cu_seqlens is not None:
        cu = cu_seqlens.tolist()
        for b in range(batch):
            a, e = cu[b], cu[b + 1]
            if e > a:
                q, k, v = qkv[a:e].float().reshape(e - a, 3, heads, Dh).permute(1, 2, 0, 3)
                p = torch.softmax((q @ k.transpose(-1, -2)) * scale, -1)
                out[a:e] = (p @ v).permute(1, 0, 2).reshape(e - a, heads * Dh).to(out.dtype)
        return out
    q, k, v = qkv.float().reshape(batch, seq, 3, heads, Dh).permute(2, 0, 3, 1, 4)
    s = (q @ k.transpose(-1, -2)) * scale
    mask = (ids.reshape(batch, 1, 1, seq) == pad_id)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    o = (p @ v).permute(0, 2, 1, 3).reshape(T, heads * Dh)
    out.copy_(o.to(out.dtype))
    return out


def cls_attention(qkv: torch.Tensor, cu_seqlens: torch.Tensor, batch: int, heads: int, scale: float | None = None,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """Attention of each packed sequence's FIRST token only (the classifier's final layer):
    ``qkv`` [T, 3*H*64] packed rows, ``cu_seqlens`` [B+1] → [B, H*64]."""
    Dh = qkv.shape[1] // (3 * heads)
    scale = (1.0 / Dh ** 0.5) if scale is None else scale
    if out is None:
        out = torch.empty((batch, heads * Dh), dtype=qkv.dtype, device=qkv.device)
    if qkv.is_cuda:
        _check(qkv, "qkv", device=qkv.device)
        _check(out, "out", device=qkv.device)
        _check(cu_seqlens, "cu_seqlens", torch.int32, qkv.device)
        _hip().cls_attention_bf16(qkv.data_ptr(), cu_seqlens.data_ptr(), out.data_ptr(), batch, heads, Dh,
                                  float(scale), _stream())
        return out
    cu = cu_seqlens.tolist()
    for b in range(batch):
        a, e = cu[b], cu[b + 1]
        if e <= a:
            out[b] = 0
            continue
        q = qkv[a, :heads * Dh].float().reshape(heads, 1, Dh)
        k = qkv[a:e, heads * Dh:2 * heads * Dh].float().reshape(e - a, heads, Dh).transpose(0, 1)
        v = qkv[a:e, 2 * heads * Dh:].float().reshape(e - a, heads, Dh).transpose(0, 1)
        p = torch.softmax((q @ k.transpose(-1, -2)) * scale, -1)
        out[b] = (p @ v).reshape(heads * Dh).to(out.dtype)
    return out


def pack_tokens(ids: torch.Tensor, pad_id: int, t_cap: int, packed: torch.Tensor, pos: torch.Tensor,
                cu: torch.Tensor, cls: torch.Tensor) -> int | None:
    """Padding-free packing of ``ids`` [B, S]: the non-pad tokens in row order into
    ``packed[:T_eff]`` (their in-row positions into ``pos``), row offsets ``cu`` [B+1] and
    the first-token row of each sequence ``cls`` [B]; ``packed[T_eff:t_cap]`` = pad.
    Device path: one kernel, no host sync (returns None); host path returns T_eff."""
    B, S = ids.shape
    if ids.is_cuda:
        for t, n in ((ids, "ids"), (packed, "packed"), (pos, "pos"), (cu, "cu"), (cls, "cls")):
            _check(t, n, torch.int32, ids.device)
        _hip().pack_tokens(ids.data_ptr(), B, S, pad_id, t_cap, packed.data_ptr(), pos.data_ptr(), cu.data_ptr(),
                           cls.data_ptr(), _stream())
        return None
    keep = ids != pad_id
    lens = keep.sum(1)
    offs = torch.zeros(B + 1, dtype=torch.int64)
    offs[1:] = torch.cumsum(lens, 0)
    n = int(offs[-1])
    if n > t_cap:
        raise ValueError(f"pack_tokens: {n} tokens exceed the capacity {t_cap}")
    packed.zero_().add_(pad_id)
    pos.zero_()
    packed[:n] = ids[keep]
    pos[:n] = torch.arange(S, dtype=torch.int32).expand(B, S)[keep]
    cu.copy_(offs.to(torch.int32))
    cls.copy_(offs[:-1].clamp(max=t_cap - 1).to(torch.int32))
    return n


def embed_layernorm(ids: torch.Tensor, type_ids: torch.Tensor | None, word: torch.Tensor, pos: torch.Tensor,
                    type_emb: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, seq: int, eps: float = 1e-12,
                    out: torch.Tensor | None = None, pos_ids: torch.Tensor | None = None) -> torch.Tensor:
    """``LN(word[ids] + pos[p] + type[type_ids])`` → [T, D] bf16 (one fused pass), with the
    position ``p = t % seq`` (padded batch) or ``pos_ids[t]`` (packed batch)."""
    T = ids.numel()
    V, D = word.shape
    if out is None:
        out = torch.empty((T, D), dtype=word.dtype, device=word.device)
    if ids.is_cuda:
        _check(ids, "ids", torch.int32, ids.device)
        for t, n in ((word, "word"), (pos, "pos"), (type_emb, "type"), (out, "out")):
            _check(t, n, device=ids.device)
        if type_ids is not None:
            _check(type_ids, "type_ids", torch.int32, ids.device)
        if pos_ids is not None:
            _check(pos_ids, "pos_ids", torch.int32, ids.device)
        if pos.shape[0] < seq:
            raise ValueError("embed_layernorm: position table shorter than the sequence")
        _hip().embed_ln_bf16(ids.data_ptr(), _ptr(type_ids), _ptr(pos_ids), word.data_ptr(), pos.data_ptr(),
                             type_emb.data_ptr(), gamma.data_ptr(), beta.data_ptr(), out.data_ptr(), T, seq, D, V,
                             float(eps), _stream())
        return out
    idx = ids.long().clamp(0, V - 1)
    p = pos_ids.long() if pos_ids is not None else torch.arange(T) % seq
    x = word.float()[idx] + pos.float()[p]
    x = x + type_emb.float()[type_ids.long() if type_ids is not None else torch.zeros(T, dtype=torch.long)]
    out.copy_(F.layer_norm(x, (D,), gamma.float(), beta.float(), eps).to(out.dtype))
    return out


# ------------------------------------------------------------------------------ layernorm
def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, residual: torch.Tensor | None = None,
              eps: float = 1e-12, out=None, sum_out=None) -> torch.Tensor:
    """``LN(x + residual)``; optionally also writes the pre-norm sum to ``sum_out``."""
    D = x.shape[-1]
    rows = x.numel() // D
    if out is None:
        out = torch.empty_like(x)
    if x.is_cuda:
        _check(x, "x", device=x.device)
        _check(out, "out", device=x.device)
        _check(gamma, "gamma", torch.float32, x.device)
        _check(beta, "beta", torch.float32, x.device)
        if residual is not None:
            _check(residual, "residual", device=x.device)
        _hip().layernorm_bf16(x.data_ptr(), _ptr(residual), gamma.data_ptr(), beta.data_ptr(), out.data_ptr(),
                              _ptr(sum_out), rows, D, float(eps), _stream())
        return out
    s = x.float() + (residual.float() if residual is not None else 0)
    if sum_out is not None:
        sum_out.copy_(s.to(sum_out.dtype))
    out.copy_(F.layer_norm(s, (D,), gamma.float(), beta.float(), eps).to(out.dtype))
    return out


# ------------------------------------------------------------------------------ direct conv
def dconv_eligible(Cin: int, KH: int, KW: int, stride, dilation, es: int, bn: int = 64) -> bool:
    """Narrow-layer direct conv (kernels/dconv.hip): stride 1/2, no dilation, Cin*es a
    multiple of the MFMA lane segment, weights + input patch within LDS."""
    sh, sw = stride
    if sh != sw or sh not in (1, 2) or tuple(dilation) != (1, 1) or KH * KW == 1:
        return False
    kl = 16 if es == 2 else 32
    if (Cin * es) % kl:
        return False
    kb = KH * KW * Cin * es
    wp = -(-kb // (4 * kl)) * (4 * kl) + 16
    ph, pw = 15 * sh + KH, 15 * sw + KW
    lds = ((ph * pw * Cin * es + 1023) & ~1023) + bn * wp + 1024
    return lds <= 96 * 1024  # leave room for >= 1 more resident workgroup


def dconv_weights(w_ohwi_bytes: torch.Tensor, Cout: int, es: int, bn: int) -> torch.Tensor:
    """[Cout, KH*KW*Cin*es] weight bytes → [round_up(Cout, bn), wp] with the kernel's pitch."""
    kl = 16 if es == 2 else 32
    kb = w_ohwi_bytes.shape[1]
    wp = -(-kb // (4 * kl)) * (4 * kl) + 16
    cpad = -(-Cout // bn) * bn
    out = torch.zeros((cpad, wp), dtype=torch.uint8, device=w_ohwi_bytes.device)
    out[:Cout, :kb] = w_ohwi_bytes
    return out


def dconv_bf16_weight_bytes(w_ohwi: torch.Tensor, bn: int) -> torch.Tensor:
    Cout = w_ohwi.shape[0]
    wb = w_ohwi.to(torch.bfloat16).contiguous().reshape(Cout, -1).view(torch.uint8)
    return dconv_weights(wb, Cout, 2, bn)


def _dconv_waves(waves, pool_rows, bn) -> int:
    """8-wave tiles pay where the filter-bank fetch dominates: BN = 64 (ResNet stem 180 -> 174 µs,
    Inception 2b 251 -> 223 µs; fp8 2b at 4 waves measured -1.7 % end to end, profiles/r05_k);
    BN = 32 tiles lose occupancy for little weight saving (2a 148 -> 156 µs) and stay at 4 waves
    (``bench/dconv_tune.py``, profiles/r02_dconv_waves)."""
    if waves is None and pool_rows is not None:
        waves = {7: 4, 14: 8}[int(pool_rows)]
    return int(waves or (8 if bn == 64 else 4))


def conv2d_direct(x: torch.Tensor, w_arr: torch.Tensor, kshape, Cout: int, bias: torch.Tensor, stride=(1, 1),
                  pad=(0, 0, 0, 0), act=None, out: torch.Tensor | None = None, out_channel_offset: int = 0,
                  bn: int = 64, chan_scale: torch.Tensor | None = None, out_scale: float | None = None,
                  maxpool_pad: tuple | None = None, pool_rows: int | None = None,
                  waves: int | None = None) -> torch.Tensor:
    """Direct conv on device: ``x`` NHWC bf16 (``chan_scale`` None) or e4m3 bytes (uint8, with
    the per-channel dequant scale ``chan_scale``); ``w_arr`` from :func:`dconv_weights`;
    ``out_scale`` → e4m3 output.  ``maxpool_pad = (top, bottom, left, right)`` fuses a 3x3 /
    stride-2 max pool of the ReLU output (ResNet stem → pool1).  ``waves`` (4 or 8, default
    default 8 for ``bn=64`` and 4 for ``bn=32``) sets the workgroup / tile size: 8 waves cover 32 x 16 conv
    pixels (pooled: 14 x 8 pooled pixels, ``pool_rows=14``; 4 waves = 16 x 16 / 7 x 8) and
    fetch the filter bank half as often; tiles whose patch would not fit LDS fall back to 4.
    Device-only (the host paths use the reference convs)."""
    N, H, W, Cin = x.shape
    KH, KW = kshape
    s = stride[0]
    pt, pb, pl, pr = pad
    Ho, Wo = conv_out_hw(H, W, KH, KW, s, s, pt, pl, 1, 1, pb, pr)
    es = 2 if x.dtype == torch.bfloat16 else 1
    out_fp8 = out_scale is not None
    Hp = Wp = ppt = ppl = 0
    oh, ow = Ho, Wo
    if maxpool_pad is not None:
        ppt, ppb, ppl, ppr = maxpool_pad
        Hp, Wp = (Ho + ppt + ppb - 3) // 2 + 1, (Wo + ppl + ppr - 3) // 2 + 1
        oh, ow = Hp, Wp
    if out is None:
        out = torch.empty((N, oh, ow, Cout), dtype=torch.uint8 if out_fp8 else torch.bfloat16, device=x.device)
        out_channel_offset = 0
    if out.shape[:3] != (N, oh, ow) or out_channel_offset + Cout > out.shape[3]:
        raise ValueError(f"conv2d_direct: out {tuple(out.shape)} cannot hold [{N},{oh},{ow},{Cout}]")
    if es == 1 and chan_scale is None:
        raise ValueError("conv2d_direct: fp8 input needs chan_scale")
    _check(x, "x", x.dtype, x.device)
    _check(w_arr, "w", torch.uint8, x.device)
    _check(bias, "bias", torch.float32, x.device)
    _check(out, "out", torch.uint8 if out_fp8 else torch.bfloat16, x.device)  # the kernel writes out_fp8 ? 1 : 2 B
    _hip().dconv(x.data_ptr(), w_arr.data_ptr(), _ptr(chan_scale), bias.data_ptr(), out.data_ptr(), es, N, H, W, Cin,
                 Cout, KH, KW, s, pt, pl, Ho, Wo, w_arr.shape[1], out.shape[3], out_channel_offset, int(out_fp8),
                 1.0 / out_scale if out_fp8 else 1.0, act_code(act), bn, _stream(), Hp, Wp, ppt, ppl,
                 _dconv_waves(waves, pool_rows, bn))
    return out


def conv2d_direct_u8s2d(x_u8: torch.Tensor, w_arr: torch.Tensor, kshape, Cout: int, bias: torch.Tensor, pad, act,
                        mean, std, out: torch.Tensor | None = None, bn: int = 64, out_scale: float | None = None,
                        waves: int | None = None) -> torch.Tensor:
    """The s2d RGB stem (``s2d_stem_weights``) straight from the raw uint8 batch ``x_u8``
    [N, Hi, Wi, 3]: the kernel builds each patch as the normalised space-to-depth rows the
    preprocess kernel would write ((v - mean) / std, no resize), so the preprocess pass and
    its bf16 tensor disappear.  ``pad``: the block-space pads; device-only."""
    N, Hi, Wi, _ = x_u8.shape
    KH, KW = kshape
    pt, pb, pl, pr = pad
    Hb, Wb = (Hi + 1) // 2, (Wi + 1) // 2
    Ho, Wo = conv_out_hw(Hb, Wb, KH, KW, 1, 1, pt, pl, 1, 1, pb, pr)
    out_fp8 = out_scale is not None
    if out is None:
        out = torch.empty((N, Ho, Wo, Cout), dtype=torch.uint8 if out_fp8 else torch.bfloat16, device=x_u8.device)
    if tuple(out.shape[:3]) != (N, Ho, Wo) or out.shape[3] < Cout:
        raise ValueError(f"conv2d_direct_u8s2d: out {tuple(out.shape)} cannot hold [{N},{Ho},{Wo},{Cout}]")
    _check(x_u8, "x", torch.uint8, x_u8.device)
    _check(w_arr, "w", torch.uint8, x_u8.device)
    _check(bias, "bias", torch.float32, x_u8.device)
    _check(out, "out", torch.uint8 if out_fp8 else torch.bfloat16, x_u8.device)
    _hip().dconv_u8s2d(x_u8.data_ptr(), w_arr.data_ptr(), bias.data_ptr(), out.data_ptr(), N, Hi, Wi, Cout, KH, KW, pt,
                       pl, Ho, Wo, w_arr.shape[1], out.shape[3], 0, int(out_fp8), 1.0 / out_scale if out_fp8 else 1.0,
                       act_code(act), bn, float(mean[0]), float(mean[1]), float(mean[2]), 1.0 / std[0], 1.0 / std[1],
                       1.0 / std[2], _stream(), _dconv_waves(waves, None, bn))
    return out


# ------------------------------------------------------------------------------ fused shortcut
def conv1x1_dual(x: torch.Tensor, x2: torch.Tensor, w_cat: torch.Tensor, bias: torch.Tensor, stride2: int = 1,
                 act=None, out: torch.Tensor | None = None, out_channel_offset: int = 0, cfg: int = -1) -> torch.Tensor:
    """``act(conv1x1(x, W[:, :K1]) + conv1x1_stride(x2, W[:, K1:]) + bias)`` in ONE K loop —
    a bottleneck's expansion conv with its projection shortcut fused (the shortcut output
    never touches HBM).  ``x`` [N,Ho,Wo,K1], ``x2`` [N,H2,W2,C2], ``w_cat`` [Cout, K1+C2]."""
    N, Ho, Wo, K1 = x.shape
    _, H2, W2, C2 = x2.shape
    Cout = w_cat.shape[0]
    if w_cat.shape[1] != K1 + C2:
        raise ValueError(f"conv1x1_dual: weights K {w_cat.shape[1]} != {K1} + {C2}")
    if out is None:
        out = torch.empty((N, Ho, Wo, Cout), dtype=x.dtype if x.is_cuda else torch.float32, device=x.device)
        out_channel_offset = 0
    a = act_code(act)
    if x.is_cuda:
        for t, n in ((x, "x"), (x2, "x2"), (w_cat, "w"), (out, "out")):
            _check(t, n, device=x.device)
        _check(bias, "bias", torch.float32, x.device)
        _hip().conv1x1_dual_bf16(x.data_ptr(), x2.data_ptr(), w_cat.data_ptr(), bias.data_ptr(), out.data_ptr(), N, Ho,
                                 Wo, K1, C2, H2, W2, stride2, Cout, out.shape[3], out_channel_offset, a, _stream(), cfg)
        return out
    xs = x2[:, ::stride2, ::stride2, :][:, :Ho, :Wo, :]
    y = x.float() @ w_cat[:, :K1].float().t() + xs.float() @ w_cat[:, K1:].float().t() + bias.float()
    out[..., out_channel_offset:out_channel_offset + Cout] = _apply_act_ref(y, a).to(out.dtype)
    return out


def pw_res_ok(K_: int, N: int, num_cu: int = 256) -> bool:
    """Shapes ``pw_res`` takes: K = 128 / 256, N in 128-channel slices, every slice group
    of the 8 XCDs resident at once."""
    return K_ in (128, 256) and N % 128 == 0 and 8 * (N // 128) <= num_cu


def pw_res(x: torch.Tensor, w_nk: torch.Tensor, bias: torch.Tensor, residual: torch.Tensor,
           out: torch.Tensor | None = None, out_channel_offset: int = 0, tp: int = 0) -> torch.Tensor:
    """``relu(x @ w^T + bias + residual)`` for a 1x1 / stride-1 expansion conv over NHWC ``x``
    ``[..., K]`` (``pw_res_ok``: K = 128 / 256, N % 128 == 0), ``w_nk`` ``[N, K]``, ``residual``
    ``[..., N]``; ``tp`` = pixels per tile for K 256 (0: the measured default, 64).
    GPU: the persistent kernel with a resident 128-channel weight slice per workgroup and
    one-tile-ahead x / residual prefetch (kernels/pw_res.hip); host: the fp32 reference."""
    K_ = x.shape[-1]
    N = w_nk.shape[0]
    lead = tuple(x.shape[:-1])
    if not pw_res_ok(K_, N) or tuple(w_nk.reshape(N, -1).shape) != (N, K_):
        raise ValueError(f"pw_res: unsupported shapes x {tuple(x.shape)}, w {tuple(w_nk.shape)}")
    if tuple(residual.shape) != (*lead, N) or bias.numel() != N:
        raise ValueError("pw_res: residual must be [..., N] and bias [N]")
    if out is None:
        out = torch.empty((*lead, N), dtype=x.dtype if x.is_cuda else torch.float32, device=x.device)
        out_channel_offset = 0
    if tuple(out.shape[:-1]) != lead or out_channel_offset + N > out.shape[-1]:
        raise ValueError(f"pw_res: out {tuple(out.shape)} cannot hold [..., {N}] at offset {out_channel_offset}")
    M = x.numel() // K_
    if x.is_cuda:
        for t, n in ((x, "x"), (w_nk, "w"), (residual, "residual"), (out, "out")):
            _check(t, n, device=x.device)
        _check(bias, "bias", torch.float32, x.device)
        dev = x.device.index if x.device.index is not None else torch.cuda.current_device()
        _hip().pw_res_bf16(x.data_ptr(), w_nk.data_ptr(), bias.data_ptr(), residual.data_ptr(), out.data_ptr(), M, N,
                           K_, out.shape[-1], out_channel_offset, residual.shape[-1], _NUM_CU[dev], _stream(), tp)
        return out
    y = x.reshape(M, K_).float() @ w_nk.reshape(N, K_).float().t() + bias.float()
    y = torch.relu(y.to(out.dtype).float() + residual.reshape(M, N).float())
    out[..., out_channel_offset:out_channel_offset + N] = y.reshape(*lead, N).to(out.dtype)
    return out


# ------------------------------------------------------------------------------ elementwise
BIN_OPS = {"add": 0, "sub": 1, "mul": 2, "div": 3, "max": 4, "min": 5, "rsub": 6, "rdiv": 7}
_BIN_REF = {0: lambda a, b: a + b, 1: lambda a, b: a - b, 2: lambda a, b: a * b, 3: lambda a, b: a / b,
            4: torch.maximum, 5: torch.minimum, 6: lambda a, b: b - a, 7: lambda a, b: b / a}


def binary(a: torch.Tensor, b, op: str, act=None, out: torch.Tensor | None = None) -> torch.Tensor:
    """``act(a OP b)`` with ``b`` a Python scalar, a fp32 vector over the last dim of ``a``,
    or a tensor of ``a``'s shape (the standalone elementwise kernel)."""
    code = BIN_OPS[op]
    a_act = act_code(act)
    if out is None:
        out = torch.empty(a.shape, dtype=a.dtype if a.is_cuda else torch.float32, device=a.device)
    if a.is_cuda:
        _check(a, "a", device=a.device)
        _check(out, "out", device=a.device)
        if isinstance(b, (int, float)):
            _hip().binary_bf16(code, a.data_ptr(), 0, out.data_ptr(), a.numel(), 0, 0, float(b), a_act, _stream())
        elif b.dim() == 1 and b.numel() == a.shape[-1]:
            _check(b, "b", torch.float32, a.device)
            _hip().binary_bf16(code, a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), 1, b.numel(), 0.0, a_act,
                               _stream())
        else:
            if tuple(b.shape) != tuple(a.shape):
                raise ValueError(f"binary: cannot broadcast {tuple(b.shape)} to {tuple(a.shape)}")
            _check(b, "b", device=a.device)
            _hip().binary_bf16(code, a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), 2, 0, 0.0, a_act, _stream())
        return out
    bb = b if isinstance(b, (int, float)) else b.float()
    out.copy_(_apply_act_ref(_BIN_REF[code](a.float(), bb if not isinstance(bb, (int, float)) else torch.tensor(bb)),
                             a_act).to(out.dtype))
    return out


def gather_rows(x: torch.Tensor, idx: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``out[r] = x[idx[r]]`` over the rows of a 2-D tensor (int32 indices; an index out of
    range gives a zero row).  On the GPU one HIP kernel (16-byte chunks), no ATen gather."""
    n = idx.numel()
    if out is None:
        out = torch.empty((n, x.shape[-1]), dtype=x.dtype, device=x.device)
    if x.is_cuda:
        _check(x, "x", x.dtype, x.device)
        _check(out, "out", x.dtype, x.device)
        _check(idx, "idx", torch.int32, x.device)
        rb = x.shape[-1] * x.element_size()
        _hip().gather_rows(x.data_ptr(), idx.data_ptr(), out.data_ptr(), n, x.shape[0], rb, _stream())
        return out
    ok = (idx >= 0) & (idx < x.shape[0])
    out.zero_()
    out[ok] = x[idx[ok].long()]
    return out


def lrn(x: torch.Tensor, depth_radius: int = 5, bias: float = 1.0, alpha: float = 1.0, beta: float = 0.5,
        out: torch.Tensor | None = None) -> torch.Tensor:
    """TF ``LRN`` on NHWC (normalisation across channels)."""
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype if x.is_cuda else torch.float32, device=x.device)
    C = x.shape[-1]
    if x.is_cuda:
        _check(x, "x", device=x.device)
        _check(out, "out", device=x.device)
        _hip().lrn_bf16(x.data_ptr(), out.data_ptr(), x.numel() // C, C, int(depth_radius), float(bias), float(alpha),
                        float(beta), _stream())
        return out
    sq = x.float() ** 2
    acc = torch.zeros_like(sq)
    for d in range(-depth_radius, depth_radius + 1):
        lo, hi = max(0, -d), min(C, C - d)
        acc[..., lo:hi] += sq[..., lo + d:hi + d]
    out.copy_((x.float() / (bias + alpha * acc) ** beta).to(out.dtype))
    return out
