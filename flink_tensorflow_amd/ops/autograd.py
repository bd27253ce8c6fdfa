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
    yf = y.float()
    if act == K.ACT_RELU:
        return (dy.float() * (yf > 0)).to(dy.dtype)
    if act == K.ACT_SIGMOID:
        return (dy.float() * yf * (1 - yf)).to(dy.dtype)
    if act == K.ACT_TANH:
        return (dy.float() * (1 - yf * yf)).to(dy.dtype)
    raise NotImplementedError(f"backward of activation {act}")


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, act):
        y = K.gemm(x, w, b, None, act)
        ctx.act = act
        ctx.save_for_backward(x, w, y)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        da = _act_grad(y, dy.contiguous(), ctx.act)
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        da2 = da.reshape(-1, da.shape[-1]).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = K.gemm(da2, w.t().contiguous()).reshape(*lead, x.shape[-1])
        if ctx.needs_input_grad[1]:
            dw = K.gemm(da2.t().contiguous(), x2.t().contiguous())
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = da2.float().sum(0)
        return dx, (dw.to(w.dtype) if dw is not None else None), db, None


def linear(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None = None, act=None) -> torch.Tensor:
    return _Linear.apply(x, w, b, K.act_code(act))


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
        w = self.weight.to(torch.bfloat16) if x.is_cuda else self.weight
        return linear(x, w, self.bias, self.act)
