"""Autograd wrappers over the hand-written MFMA training GEMM (online-training path).

``linear(x, w, b, act)`` computes ``act(x @ w^T + b)``; on the GPU all three GEMMs of the
layer run on ``kernels/gemm_train.hip`` (``ops.kernels.gemm_train``), none on a library:

* forward  y  = act(x · Wᵀ + b)      gemm_train(x, W)            fused bias + activation
* dact     = dy * act'(y)            elementwise, from the saved output (ReLU / sigmoid / tanh)
* dx       = dact · W                gemm_train(dact, W, w_t)    W read K-major (transpose reads)
* dW       = dactᵀ · x               gemm_train(dact, x, x_t, w_t) fp32 result for the fp32 master
* db       = Σ_rows dact             fp32 column sum

Shapes the kernel does not take (K or N not a multiple of 8) use the older igemm forward
and fp32 host-reference GEMMs; on host tensors the same math runs in fp32.
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


def _train_ok(x2: torch.Tensor, wc: torch.Tensor) -> bool:
    return (x2.is_cuda and x2.dtype == torch.bfloat16 and wc.dtype == torch.bfloat16 and x2.shape[1] % 8 == 0
            and wc.shape[0] % 8 == 0)


class _Linear(torch.autograd.Function):
    """Forward and backward on the layout-general MFMA training GEMM (no transposed copies,
    fp32 weight gradient written by the GEMM itself, no cast kernels)."""

    @staticmethod
    def forward(ctx, x, w, w_compute, b, act):
        lead = x.shape[:-1]
        x2 = x.reshape(-1, x.shape[-1])
        if _train_ok(x2, w_compute):
            x2 = x2 if x2.stride(1) == 1 else x2.contiguous()
            y = K.gemm_train(x2, w_compute, bias=b, act=act).reshape(*lead, w_compute.shape[0])
        else:
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
        gpu = _train_ok(x2, wc)
        if gpu:
            da2 = da2.to(torch.bfloat16)
            da2 = da2 if da2.stride(1) == 1 else da2.contiguous()
            x2 = x2 if x2.stride(1) == 1 else x2.contiguous()
        if ctx.needs_input_grad[0]:
            if gpu:
                dx = K.gemm_train(da2, wc, w_t=True).to(x.dtype).reshape(*lead, x.shape[-1])
            else:
                dx = (da2.float() @ wc.float()).to(x.dtype).reshape(*lead, x.shape[-1])
        if ctx.needs_input_grad[1]:
            if gpu:
                dw = K.gemm_train(da2, x2, x_t=True, w_t=True, out_dtype=torch.float32).to(ctx.w_dtype)
            else:
                dw = (da2.float().t() @ x2.float()).to(ctx.w_dtype)
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
