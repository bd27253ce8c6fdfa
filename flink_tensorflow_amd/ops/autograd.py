"""Autograd wrappers over the MFMA GEMM kernel (online-training path).

``linear(x, w, b, act)`` computes ``act(x @ w^T + b)`` with the fused-epilogue GEMM in the
forward pass; the backward pass is three more MFMA GEMM launches:

* dact  = dy * act'(pre)   (elementwise, recomputed from the saved output for ReLU/sigmoid)
* dx    = dact · W         → gemm(dact[M,N], W^T[K,N])
* dW    = dactᵀ · x        → gemm(dactᵀ[N,M], xᵀ[K,M])
* db    = Σ_rows dact

On host tensors the same math runs through the fp32 reference ops.
"""
from __future__ import annotations

import torch

from . import kernels as K


def _act_grad(y: torch.Tensor, dy: torch.Tensor, act: int) -> torch.Tensor:
    if act == K.ACT_NONE:
        return dy
    if act == K.ACT_RELU:
        return dy * (y > 0)
    yf = y.float()
    if act == K.ACT_SIGMOID:
        return (dy.float() * yf * (1 - yf)).to(dy.dtype)
    if act == K.ACT_TANH:
        return (dy.float() * (1 - yf * yf)).to(dy.dtype)
    raise NotImplementedError(f"backward of activation {act}")


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a @ b`` with an fp32 result: bf16 operands accumulate in fp32 and are written as
    fp32 by the library GEMM itself (no bf16 rounding of the weight gradient, no cast)."""
    if a.is_cuda and a.dtype != torch.float32:
        return torch.mm(a, b, out_dtype=torch.float32)
    return torch.mm(a.float(), b.float())


class _Linear(torch.autograd.Function):
    """Forward on the hand-written MFMA GEMM with the fused bias + activation epilogue.
    Backward: the activation mask, then two plain GEMMs on the library (dX = dA.W, NN;
    dW = dA^T.X, TN with an fp32 result for the fp32 master weight — no transposed copies,
    no cast kernels) and the bias gradient as one fp32 column sum."""

    @staticmethod
    def forward(ctx, x, w, w_compute, b, act):
        y = K.gemm(x, w_compute, b, None, act)
        ctx.act = act
        ctx.w_dtype = w.dtype
        ctx.save_for_backward(x, w_compute, y)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wc, y = ctx.saved_tensors
        da = _act_grad(y, dy, ctx.act)
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        da2 = da.reshape(-1, da.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(da2.to(wc.dtype), wc).to(x.dtype).reshape(*lead, x.shape[-1])
        if ctx.needs_input_grad[1]:
            dw = _mm_f32(da2.t(), x2).to(ctx.w_dtype)
        if ctx.has_b and ctx.needs_input_grad[3]:
            db = da2.sum(0, dtype=torch.float32)
        return dx, dw, None, db, None


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act=None,
           w_compute: torch.Tensor | None = None) -> torch.Tensor:
    """``act(x @ w^T + b)``; ``w_compute``: the operand the GEMMs read (e.g. a bf16 copy of
    an fp32 master ``w``, which receives the fp32 gradient)."""
    return _Linear.apply(x, w, w if w_compute is None else w_compute, b, K.act_code(act))


class Linear(torch.nn.Module):
    """fp32 master weights [out, in] + fp32 bias; on the GPU the forward casts the weights
    to bf16 for the MFMA GEMM (the cast's backward returns fp32 gradients), so optimizers
    update full-precision weights."""

    def __init__(self, in_features: int, out_features: int, act=None, bias: bool = True, dtype=torch.float32,
                 device=None):
        super().__init__()
        w = torch.empty(out_features, in_features, dtype=torch.float32)
        torch.nn.init.kaiming_uniform_(w, a=5 ** 0.5)
        self.weight = torch.nn.Parameter(w.to(device))
        self.bias = torch.nn.Parameter(torch.zeros(out_features, dtype=torch.float32, device=device)) if bias else None
        self.act = K.act_code(act)
        self.compute_dtype = dtype

    def forward(self, x):
        if not x.is_cuda:
            return linear(x, self.weight, self.bias, self.act)
        with torch.no_grad():  # the bf16 operand is a copy, outside autograd: dW lands on the master
            w16 = self.weight.to(torch.bfloat16)
        return linear(x, self.weight, self.bias, self.act, w_compute=w16)
