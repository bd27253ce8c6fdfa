"""Layout-general training GEMM (``kernels/gemm_train.hip``) against a PyTorch fp32
reference: forward NT, dX = dA W (W K-major), dW = dA^T H (both K-major) on the Wide&Deep
shapes (4096 x {1024, 512, 256}), M / N tails, split-K, and the bf16 epilogues."""
import pytest
import torch

from flink_tensorflow_amd.ops import kernels as K

SHAPES = [  # (M, N, K)
    (4096, 1024, 896), (4096, 512, 1024), (4096, 256, 512),     # forward / dX
    (1024, 896, 4096), (512, 1024, 4096), (256, 512, 4096),     # dW (K = batch)
    (200, 72, 192),                                             # tails
]


def _ref(x, w, x_t, w_t):
    X = x.float().t() if x_t else x.float()
    W = w.float() if w_t else w.float().t()
    return X @ W


def _operands(M, N, Kd, x_t, w_t, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn((Kd, M) if x_t else (M, Kd), generator=g).to(torch.bfloat16).to(dev)
    w = torch.randn((Kd, N) if w_t else (N, Kd), generator=g).to(torch.bfloat16).to(dev)
    return x, w


def test_gemm_train_cpu_reference_layouts():
    x, w = _operands(48, 40, 64, True, True, "cpu")
    y = K.gemm_train(x, w, x_t=True, w_t=True, out_dtype=torch.float32)
    torch.testing.assert_close(y, x.float().t() @ w.float(), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("x_t,w_t", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("shape", SHAPES)
def test_gemm_train_layouts_fp32_out_gpu(shape, x_t, w_t):
    M, N, Kd = shape
    dev = torch.device("cuda", 0)
    x, w = _operands(M, N, Kd, x_t, w_t, dev)
    y = K.gemm_train(x, w, x_t=x_t, w_t=w_t, out_dtype=torch.float32)
    ref = _ref(x, w, x_t, w_t)
    err = (y - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-3, (shape, x_t, w_t, err)


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [1, 3, 8])
def test_gemm_train_split_k_gpu(splits):
    dev = torch.device("cuda", 0)
    x, w = _operands(256, 512, 4096, True, True, dev, seed=1)
    y = K.gemm_train(x, w, x_t=True, w_t=True, out_dtype=torch.float32, splits=splits)
    ref = _ref(x, w, True, True)
    assert (y - ref).abs().max().item() / ref.abs().max().item() < 2e-3
    y2 = K.gemm_train(x, w, x_t=True, w_t=True, out_dtype=torch.float32, splits=splits)
    assert torch.equal(y, y2)  # fixed-order reduction: deterministic


@pytest.mark.gpu
@pytest.mark.parametrize("splits", [1, 4])
def test_gemm_train_bf16_epilogues_gpu(splits):
    dev = torch.device("cuda", 0)
    M, N, Kd = 4096, 512, 1024
    x, w = _operands(M, N, Kd, False, False, dev, seed=2)
    bias = torch.randn(N, device=dev)
    y = K.gemm_train(x, w, bias=bias, act="relu", splits=splits)
    ref = torch.relu(x.float() @ w.float().t() + bias)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    # dX with the ReLU backward mask of the layer input, written into a row-strided view
    dA, W = _operands(M, N, Kd, False, True, dev, seed=3)
    mask = torch.randn(M, N, device=dev).to(torch.bfloat16)
    big = torch.zeros(M, N + 64, dtype=torch.bfloat16, device=dev)
    K.gemm_train(dA, W, w_t=True, mask=mask, out=big[:, :N], splits=splits)
    ref = torch.where(mask.float() > 0, dA.float() @ W.float(), torch.zeros(M, N, device=dev))
    torch.testing.assert_close(big[:, :N].float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    assert big[:, N:].abs().sum() == 0


@pytest.mark.gpu
def test_gemm_train_cost_model_splits_deep_k():
    assert K.gemm_train_splits(1024, 896, 4096) > 1   # 56 tiles over 256 CUs: split
    assert K.gemm_train_splits(4096, 1024, 896) == 1  # 256 tiles: no split
